"""Build the native library dccrg_amd/libdccrgx.so (hipcc, gfx950) in-tree.

The .so links RCCL and the HIP runtime by soname (libamdhip64.so.7,
librccl.so.1); when it is loaded into a process that already holds
PyTorch's copies of those libraries, the dynamic loader reuses them, so the
library and torch share one HIP runtime.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libdccrgx.so")
SOURCES = ["api.hip", "grid.hip", "mesh.hip", "comm.hip", "partition.hip", "build_kernels.hip", "tile_build.hip", "sweep_kernels.hip",
           "poisson_kernels.hip", "gol_amr.hip", "varfield.hip", "pool.hip"]
HEADERS = ["dccrgx_internal.hpp", "dccrgx_grid.hpp", "dccrgx_mapping.hpp", "dccrgx_mesh.hpp", "dccrgx_neighbors.hpp"]
ARCH = os.environ.get("DCCRGX_ARCH", "gfx950")


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(os.path.dirname(HERE), "include", "dccrgx.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False, out=None, defines=()):
    """Compile every source and link OUT.  `out` / `defines` build an
    experiment variant next to it (e.g. libdccrgx_b.so with -DNAME=1) for a
    paired A/B; the product always loads OUT."""
    if out is None and not force and not _stale():
        return OUT
    out = out or OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objs = []
    procs = []
    for src in SOURCES:
        obj = os.path.join(CSRC, src.replace(".hip", ".o"))
        obj = obj.replace(".o", f".{os.path.basename(out)}.o")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC"] + [f"-D{d}" for d in defines] + [
               "-c", os.path.join(CSRC, src), "-o", obj,
               "-Wall", "-Wno-unused-function", "-Wno-unused-parameter", "-Wno-pass-failed"]
        if verbose:
            print(" ".join(cmd))
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    for p in procs:
        if p.wait() != 0:
            raise RuntimeError("hipcc failed")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs + [
        "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    for o in objs:
        os.remove(o)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(OUT)
