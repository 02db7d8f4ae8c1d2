"""Build the in-tree native extensions for MI355X (gfx950).

Compiles every ``csrc/kernels/*.hip`` with ``hipcc --offload-arch=gfx950`` into objects, links
them with the pybind11 bindings into ``fraud_detection_amd/_fdx_native*.so``, and (separately)
builds the RCCL communicator ``_fdx_comm*.so`` and the native CSV reader ``_fdx_io*.so``.  The
shared objects stay inside the package directory (they travel to the GPU box with the repo
snapshot) and carry an RPATH to torch's bundled ROCm libraries: torch ships
``libamdhip64.so.7`` / ``librccl.so.1`` with the same SONAMEs as /opt/rocm, so importing torch
first makes our extension bind to the SAME HIP runtime instance (one HIP context per process).

Incremental: an object is rebuilt only when its source or any header is newer.
Usage:  python -m fraud_detection_amd.build_native [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD = os.path.join(PKG_DIR, "csrc", "build")
ARCH = os.environ.get("FDX_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _torch_lib_dir() -> str:
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return os.path.join(ROCM, "lib")
    return os.path.join(os.path.dirname(spec.origin), "lib")


def _py_includes() -> list[str]:
    import pybind11

    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + res.stdout + res.stderr)
        raise RuntimeError(f"native build step failed: {os.path.basename(cmd[-1])}")


COMMON_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]
# Per-file code generation options.  knn.hip: MFMA accumulators in arch VGPRs (gfx950's unified
# register file) -- its 16-float score tile is consumed by VALU right after every MFMA chain, and
# the AGPR form costs 32 v_accvgpr moves per 32x32 tile.
# kernelshap.hip: same reasoning -- every MFMA tile feeds the sigmoid epilogue directly; and no SLP
# packing of its scalar f32 epilogue into v_pk_*_f32 (no faster than two plain ops, dearer beside MFMAs).
PER_FILE_FLAGS = {"knn.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
                  "kernelshap.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1", "-fno-slp-vectorize"]}


def _compile(src: str, obj: str, headers: list[str], force: bool, extra: list[str]) -> str:
    if force or _newer(obj, [src] + headers):
        cmd = [HIPCC, f"--offload-arch={ARCH}", *COMMON_FLAGS, *extra, "-c", src, "-o", obj]
        _run(cmd)
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> dict:
    os.makedirs(BUILD, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    kern_srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    jobs = jobs or min(8, os.cpu_count() or 4)
    inc = [f"-I{CSRC}", f"-I{os.path.join(CSRC, 'kernels')}"]
    tasks = []
    for src in kern_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        tasks.append((src, obj, inc + PER_FILE_FLAGS.get(os.path.basename(src), [])))
    bind_src = os.path.join(CSRC, "bindings.cpp")
    tasks.append((bind_src, os.path.join(BUILD, "bindings.o"), inc + _py_includes()))
    comm_src = os.path.join(CSRC, "comm", "rccl_comm.cpp")
    io_src = os.path.join(CSRC, "io", "csv_reader.cpp")
    if os.path.exists(comm_src):
        tasks.append((comm_src, os.path.join(BUILD, "rccl_comm.o"), inc + _py_includes() + [f"-I{ROCM}/include"]))
    if os.path.exists(io_src):
        tasks.append((io_src, os.path.join(BUILD, "csv_reader.o"), inc + _py_includes()))
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_compile, s, o, headers, force, e) for (s, o, e) in tasks]
        objs = [f.result() for f in futs]
    torch_lib = _torch_lib_dir()
    rpath = [f"-Wl,-rpath,{torch_lib}", f"-Wl,-rpath,{ROCM}/lib"]
    outputs = {}
    kern_objs = [o for o in objs if os.path.basename(o).endswith(".hip.o")] + [os.path.join(BUILD, "bindings.o")]
    native = os.path.join(PKG_DIR, "_fdx_native" + EXT_SUFFIX)
    if force or _newer(native, kern_objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *kern_objs, "-o", native, *rpath])
    outputs["native"] = native
    comm_obj = os.path.join(BUILD, "rccl_comm.o")
    if os.path.exists(comm_obj):
        comm = os.path.join(PKG_DIR, "_fdx_comm" + EXT_SUFFIX)
        if force or _newer(comm, [comm_obj]):
            _run([HIPCC, "-shared", "-fPIC", comm_obj, "-o", comm, f"-L{ROCM}/lib", "-lrccl", *rpath])
        outputs["comm"] = comm
    io_obj = os.path.join(BUILD, "csv_reader.o")
    if os.path.exists(io_obj):
        io = os.path.join(PKG_DIR, "_fdx_io" + EXT_SUFFIX)
        if force or _newer(io, [io_obj]):
            _run([HIPCC, "-shared", "-fPIC", io_obj, "-o", io, "-lpthread", *rpath])
        outputs["io"] = io
    # the serving ring is host-only C++ (front-end processes import it without any HIP runtime)
    ring_src = os.path.join(CSRC, "serve", "shm_ring.cpp")
    if os.path.exists(ring_src):
        ring = os.path.join(PKG_DIR, "_fdx_ring" + EXT_SUFFIX)
        if force or _newer(ring, [ring_src, os.path.join(CSRC, "serve", "shm_ring.h")]):
            _run([os.environ.get("CXX", "g++"), *COMMON_FLAGS, "-shared", *_py_includes(), ring_src, "-o", ring,
                  "-lpthread"])
        outputs["ring"] = ring
    if verbose:
        for k, v in outputs.items():
            print(f"[build_native] {k}: {os.path.relpath(v, os.path.dirname(PKG_DIR))}")
    return outputs


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs, verbose=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
