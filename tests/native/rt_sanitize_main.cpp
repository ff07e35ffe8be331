// AddressSanitizer + UndefinedBehaviorSanitizer harness for the host runtime
// (SURVEY §5.2). The runtime sources are compiled INTO this executable with
// -fsanitize=address,undefined and exposed to an embedded CPython as module
// `_rt_san`; tests/native/rt_stress.py then drives them. Because the
// sanitizer runtime is part of the main executable, no preload is needed.
// Usage: rt_sanitize <path/to/rt_stress.py>
#include <pybind11/embed.h>

#include <cstdio>
#include <string>

namespace py = pybind11;

void register_block_manager(py::module_& m);
void register_kv_index(py::module_& m);
void register_gbdt(py::module_& m);
void register_fs_store(py::module_& m);
void register_epp_score(py::module_& m);

PYBIND11_EMBEDDED_MODULE(_rt_san, m) {
  register_block_manager(m);
  register_kv_index(m);
  register_gbdt(m);
  register_fs_store(m);
  register_epp_score(m);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s rt_stress.py\n", argv[0]);
    return 2;
  }
  py::scoped_interpreter guard;
  try {
    py::module_ sys = py::module_::import("sys");
    std::string script = argv[1];
    sys.attr("path").attr("insert")(0, script.substr(0, script.find_last_of('/')));
    py::module_ drv = py::module_::import("rt_stress");
    py::object res = drv.attr("run_all")(py::module_::import("_rt_san"));
    std::printf("rt_sanitize ok: %s\n", std::string(py::str(res)).c_str());
  } catch (const std::exception& e) {
    std::fprintf(stderr, "rt_sanitize failed: %s\n", e.what());
    return 1;
  }
  return 0;
}
