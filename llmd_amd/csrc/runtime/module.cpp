// pybind11 module for the llmd_amd host runtime (`llmd_amd._rt`).
#include <pybind11/pybind11.h>

namespace py = pybind11;

void register_block_manager(py::module_& m);
void register_kv_index(py::module_& m);
void register_gbdt(py::module_& m);
void register_fs_store(py::module_& m);
void register_shm_ring(py::module_& m);
void register_epp_score(py::module_& m);

PYBIND11_MODULE(_rt, m) {
  m.doc() = "llmd_amd native host runtime";
  register_block_manager(m);
  register_kv_index(m);
  register_gbdt(m);
  register_fs_store(m);
  register_shm_ring(m);
  register_epp_score(m);
}
