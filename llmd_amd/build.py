"""In-tree native build for llmd_amd (no JIT cache, no hipify).

Two extension modules are produced next to this file:

* ``_C``  - the HIP/CDNA4 op library: every ``csrc/ops/*.hip`` compiled by
  ``hipcc --offload-arch=gfx950`` plus ``csrc/ops/bindings.cpp`` (torch
  pybind11 bindings) compiled by g++, linked against torch's own HIP runtime.
* ``_rt`` - the host C++ runtime (block manager / prefix cache, KV-event
  index, GBDT latency predictor, offload/FS tier, ...): ``csrc/runtime/*.cpp``
  with pybind11 only (no torch, no HIP), so CPU-only hosts can use it.

Objects are cached by a content hash of (source, headers, flags), so a rebuild
only recompiles what changed. ``python -m llmd_amd.build`` builds both.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "llmd_native"
ARCH = os.environ.get("LLMD_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _torch_paths():
    import torch.utils.cpp_extension as ce  # noqa: WPS433

    inc = ce.include_paths()
    lib = ce.library_paths()[0]
    return inc, lib


def _pybind_inc():
    import pybind11

    return pybind11.get_include()


def _py_inc():
    return sysconfig.get_paths()["include"]


def _hash(paths, flags):
    h = hashlib.sha256()
    for p in paths:
        h.update(Path(p).read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _headers(d: Path):
    return sorted(str(p) for p in d.rglob("*.h"))


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def _compile(src: Path, cmd_prefix, flags, deps, out_dir: Path):
    key = _hash([src] + deps, cmd_prefix + flags)
    obj = out_dir / f"{src.stem}.{key}.o"
    if not obj.exists():
        tmp = obj.with_suffix(".tmp.o")
        _run(cmd_prefix + flags + ["-c", str(src), "-o", str(tmp)])
        os.replace(tmp, obj)
    return obj


def _link(objs, out: Path, libs):
    key = _hash(objs, libs)
    stamp = out.with_name(out.name + ".stamp")
    if out.exists() and stamp.exists() and stamp.read_text() == key:
        return out
    tmp = out.with_name(out.name + ".tmp")
    _run(["g++", "-shared", "-o", str(tmp)] + [str(o) for o in objs] + libs)
    os.replace(tmp, out)
    stamp.write_text(key)
    return out


def build_ops(jobs: int = 8, verbose: bool = False, debug: bool = False) -> Path:
    """Build the HIP op library ``llmd_amd/_C`` - or, with ``debug``,
    ``llmd_amd/_C_debug``: -O1 -g kernels with the LLMD_DCHECK device
    assertions compiled in (SURVEY §5.2 debug kernel build; select it at run
    time with LLMD_KERNEL_DEBUG=1, best together with AMD_SERIALIZE_KERNEL=3)."""
    tinc, tlib = _torch_paths()
    name = "_C_debug" if debug else "_C"
    out_dir = BUILD / ("ops_debug" if debug else "ops")
    out_dir.mkdir(parents=True, exist_ok=True)
    inc = CSRC / "include"
    deps = _headers(inc) + sorted(str(p) for p in (CSRC / "ops").glob("*.inc"))  # + generated asm includes
    hip_srcs = sorted((CSRC / "ops").glob("*.hip"))
    hip_flags = [
        f"--offload-arch={ARCH}", "-O1" if debug else "-O3", "-fPIC", "-std=c++17", f"-I{inc}",
        "-ffp-contract=fast", "-munsafe-fp-atomics",
    ] + (["-g", "-DLLMD_KERNEL_DEBUG=1"] if debug else [])
    cpp_flags = [
        "-O2", "-fPIC", "-std=c++17", f"-I{inc}", f"-I{ROCM}/include", f"-I{_py_inc()}",
        "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-DTORCH_EXTENSION_NAME={name}",
        "-DTORCH_API_INCLUDE_EXTENSION_H", "-D_GLIBCXX_USE_CXX11_ABI=1", "-w",
    ] + [f"-I{p}" for p in tinc]
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, s, [f"{ROCM}/bin/hipcc"], hip_flags, deps, out_dir) for s in hip_srcs]
        futs.append(ex.submit(_compile, CSRC / "ops" / "bindings.cpp", ["g++"], cpp_flags, deps, out_dir))
        objs = [f.result() for f in futs]
    libs = [
        f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
        "-ltorch_python", "-lamdhip64", f"-Wl,-rpath,{tlib}",
    ]
    out = _link(objs, PKG / f"{name}{EXT}", libs)
    _check_launch_stubs(out)
    if verbose:
        print(f"[llmd build] {out}")
    return out


def _check_launch_stubs(lib: Path) -> None:
    """Fail the build when a kernel's host launch stub is missing from the library: the link of a
    shared object leaves it undefined and the failure would only show at import time on the GPU box
    (hipcc's host pass drops the stub of a kernel template whose DMA lambda reads an array of
    template-dependent size - seen in moe4.hip)."""
    try:
        r = subprocess.run(["nm", "-D", "--undefined-only", str(lib)], capture_output=True, text=True, check=True)
    except (OSError, subprocess.CalledProcessError):
        return  # no binutils: the import check of __graft_entry__.build() still catches it
    # the stub is named __device_stub__<kernel> or, for a kernel in an anonymous namespace, after the kernel
    # itself (_ZN12_GLOBAL__N_...): a library's own anonymous-namespace symbol is never legitimately external
    missing = [l.split()[-1] for l in r.stdout.splitlines() if "__device_stub__" in l or "_GLOBAL__N_" in l]
    if missing:
        raise RuntimeError(f"{lib.name}: {len(missing)} kernel launch stubs undefined, e.g. {missing[0]}")


def build_runtime(jobs: int = 8, verbose: bool = False) -> Path:
    """Build the host C++ runtime ``llmd_amd/_rt`` (pybind11, no torch/HIP)."""
    out_dir = BUILD / "rt"
    out_dir.mkdir(parents=True, exist_ok=True)
    rdir = CSRC / "runtime"
    deps = _headers(rdir) + _headers(CSRC / "include")
    srcs = sorted(rdir.glob("*.cpp"))
    flags = ["-O3", "-fPIC", "-std=c++17", f"-I{rdir}", f"-I{_pybind_inc()}", f"-I{_py_inc()}",
             "-fvisibility=hidden", "-pthread"]
    extra = os.environ.get("LLMD_RT_CFLAGS", "").split()
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, ["g++"], flags + extra, deps, out_dir), srcs))
    return _link(objs, PKG / f"_rt{EXT}", ["-pthread"] + extra)


def build_sanitized_runtime(verbose: bool = False) -> Path:
    """ASan+UBSan executable embedding CPython with the runtime compiled in
    (tests/native/rt_sanitize_main.cpp). Host code only - GPU
    sanitizers are not used."""
    rdir = CSRC / "runtime"
    srcs = [s for s in sorted(rdir.glob("*.cpp")) if s.name != "module.cpp"]
    main = PKG.parent / "tests" / "native" / "rt_sanitize_main.cpp"
    out = BUILD / "rt_sanitize"
    BUILD.mkdir(parents=True, exist_ok=True)
    libdir = sysconfig.get_config_var("LIBDIR")
    ver = sysconfig.get_config_var("LDVERSION")
    flags = ["-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
             "-fno-sanitize-recover=undefined", f"-I{rdir}", f"-I{_pybind_inc()}", f"-I{_py_inc()}", "-pthread"]
    odir = BUILD / "rt_san"
    odir.mkdir(parents=True, exist_ok=True)
    deps = _headers(rdir)
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        objs = list(ex.map(lambda src: _compile(src, ["g++"], flags, deps, odir), srcs + [main]))
    key = _hash(objs, flags)
    stamp = out.with_name(out.name + ".stamp")
    if out.exists() and stamp.exists() and stamp.read_text() == key:
        return out
    _run(["g++", "-fsanitize=address,undefined", "-pthread"] + [str(o) for o in objs] +
         ["-o", str(out), f"-L{libdir}", f"-lpython{ver}", f"-Wl,-rpath,{libdir}"])
    stamp.write_text(key)
    if verbose:
        print(f"[llmd build] {out}")
    return out


RELAY = PKG / "bin" / "llmd-relay"


def build_relay(verbose: bool = False) -> Path:
    """The router's native data plane (``csrc/relay/relay.cpp``, router/relay.py): a
    standalone epoll executable, no Python / torch / HIP."""
    src = CSRC / "relay" / "relay.cpp"
    flags = ["-O2", "-std=c++17", "-pthread", "-Wall"]
    key = _hash([src], flags)
    stamp = RELAY.with_name(RELAY.name + ".stamp")
    if RELAY.exists() and stamp.exists() and stamp.read_text() == key:
        return RELAY
    RELAY.parent.mkdir(parents=True, exist_ok=True)
    tmp = RELAY.with_name(RELAY.name + ".tmp")
    _run(["g++"] + flags + [str(src), "-o", str(tmp)])
    os.replace(tmp, RELAY)
    stamp.write_text(key)
    if verbose:
        print(f"[llmd build] {RELAY}")
    return RELAY


def build_all(jobs: int | None = None, verbose: bool = True):
    jobs = jobs or min(8, os.cpu_count() or 4)
    build_relay(verbose)
    rt = build_runtime(jobs, verbose)
    ops = build_ops(jobs, verbose)
    if verbose:
        print(f"[llmd build] ok: {rt.name} {ops.name}")
    return rt, ops


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what == "ops":
        build_ops(verbose=True)
    elif what == "rt":
        build_runtime(verbose=True)
    elif what == "relay":
        build_relay(verbose=True)
    elif what == "sanitize":
        build_sanitized_runtime(verbose=True)
    elif what == "debug":
        build_ops(verbose=True, debug=True)
    else:
        build_all()
