"""In-tree native build for parameter_server_amd.

Builds two shared objects next to this file (so they travel with the repo
snapshot to a GPU box and are visibly loaded from the tree):

* ``_hipops.so``  -- hand-written HIP kernels for gfx950 (``csrc/hip/*.hip``)
  plus their torch/pybind11 bindings (``csrc/hip/bind.cpp``). Compiled directly
  with ``hipcc --offload-arch=gfx950`` (no hipify step, no CUDA sources).
* ``_pscore.so``  -- the host C++ runtime (``csrc/core/*.cc``): TCP van,
  protobuf-text config parser, data parsers, RecordIO, crc32c/murmur3,
  CountMin/Bloom/Bitmap, CPU reference kernels. Pure C++17 + pybind11; it does
  not depend on torch so it builds in seconds.

Incremental: an object is rebuilt only when its source or any header in its
directory is newer. Run ``python -m parameter_server_amd._build``.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "native"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
CXX = shutil.which("g++") or "c++"


def _py_includes() -> list[str]:
    import pybind11

    return [sysconfig.get_paths()["include"], pybind11.get_include()]


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce

    inc = ce.include_paths(device_type="cuda")
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _stale(obj: Path, src: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(p.stat().st_mtime > t for p in [src, *deps])


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build_hipops(jobs: int = 8, verbose: bool = False) -> Path:
    inc, torch_lib, abi = _torch_paths()
    src_dir = CSRC / "hip"
    out_dir = BUILD / "hip"
    out_dir.mkdir(parents=True, exist_ok=True)
    headers = sorted(src_dir.glob("*.cuh")) + sorted(src_dir.glob("*.h"))
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", str(src_dir),
              "-Wno-unused-result", "-Wno-deprecated-declarations"]
    jobs_list = []
    objs = []
    for src in sorted(src_dir.glob("*.hip")):
        obj = out_dir / (src.stem + ".o")
        objs.append(obj)
        if _stale(obj, src, headers):
            jobs_list.append([HIPCC, *common, "-c", str(src), "-o", str(obj)])
    bind = src_dir / "bind.cpp"
    bobj = out_dir / "bind.o"
    objs.append(bobj)
    if _stale(bobj, bind, headers):
        tflags = [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_hipops",
                  "-DTORCH_API_INCLUDE_EXTENSION_H", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1"]
        incs = sum((["-isystem", p] for p in inc + _py_includes()), [])
        jobs_list.append([HIPCC, *common, *tflags, *incs, "-x", "hip", "-c", str(bind),
                          "-o", str(bobj)])
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_run, c) for c in jobs_list]
        for c, f in zip(jobs_list, futs):
            if verbose:
                print("[hipcc]", Path(c[c.index("-c") + 1]).name, flush=True)
            f.result()
    target = PKG / "_hipops.so"
    if jobs_list or not target.exists():
        libs = ["-L", torch_lib, "-Wl,-rpath," + torch_lib, "-lc10", "-lc10_hip", "-ltorch",
                "-ltorch_cpu", "-ltorch_hip", "-ltorch_python"]
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o",
              str(target), *libs])
    return target


def build_pscore(jobs: int = 8, verbose: bool = False) -> Path | None:
    src_dir = CSRC / "core"
    srcs = sorted(src_dir.glob("*.cc"))
    if not srcs:
        return None
    out_dir = BUILD / "core"
    out_dir.mkdir(parents=True, exist_ok=True)
    headers = sorted(src_dir.glob("*.h"))
    flags = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-pthread",
             "-fvisibility=hidden", "-I", str(src_dir)] + sum((["-isystem", p] for p in _py_includes()), [])
    objs, jobs_list = [], []
    for src in srcs:
        obj = out_dir / (src.stem + ".o")
        objs.append(obj)
        if _stale(obj, src, headers):
            jobs_list.append([CXX, *flags, "-c", str(src), "-o", str(obj)])
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for c, f in zip(jobs_list, [ex.submit(_run, c) for c in jobs_list]):
            if verbose:
                print("[c++]", Path(c[c.index("-c") + 1]).name, flush=True)
            f.result()
    target = PKG / ("_pscore" + sysconfig.get_config_var("EXT_SUFFIX"))
    if jobs_list or not target.exists():
        _run([CXX, "-shared", "-pthread", *map(str, objs), "-o", str(target), "-lz"])
    return target


def build_all(verbose: bool = True) -> None:
    jobs = int(os.environ.get("MAX_JOBS", "8"))
    p = build_pscore(jobs, verbose)
    if verbose and p:
        print("built", p.name)
    h = build_hipops(jobs, verbose)
    if verbose:
        print("built", h.name)


if __name__ == "__main__":
    build_all(verbose="-q" not in sys.argv)
