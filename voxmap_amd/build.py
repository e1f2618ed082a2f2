"""In-tree build of libvoxmap_hip.so for gfx950 (hipcc, no JIT cache).

Flags that are part of the numerical contract:
  -ffp-contract=off      no FMA contraction (HIP's default is fast-honor-pragmas)
  (default) -fhip-fp32-correctly-rounded-divide-sqrt  IEEE fp32 / and sqrt
(-fno-slp-vectorize is a speed flag: it does not change fp32 results.)
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libvoxmap_hip.so")
# the render kernel's EXT modes compile in units of their own (vx_render.h), listed
# first: they are the long ones, and the pool starts them first
SOURCES = ["vx_render_e56.hip", "vx_render_e2.hip", "vx_render_e1.hip", "vx_render_e0.hip", "vx_render_e3.hip",
           "vx_render_e4.hip", "vx_kernels.hip", "vx_field_gpu.hip", "vx_api.cpp", "vx_host.cpp", "vx_codec.cpp",
           "vx_field.cpp", "vx_frame.cpp", "vx_mgpu.cpp"]
HEADERS = ["vx_internal.h", "vx_render.h"]
ARCH = os.environ.get("VOXMAP_ARCH", "gfx950")
# -fno-slp-vectorize: packed FP32 (v_pk_*) issues at the cost of two scalar ops
# on gfx950 (profiles/r01_valu_costs.txt), so SLP packing only adds moves.
# -instcombine-max-copied-from-constant-users: the render kernels take KernelArgs
# by value and read it through ~300+ pointers; past LLVM's default limit (300)
# InstCombine stops replacing the kernel's private copy of the arguments by the
# kernarg segment itself and every lane copies 1.5 KB to scratch
# (kernel_meta.check catches that).  A speed flag: no effect on fp32 results.
FLAGS = ["-O3", "-std=c++20", "-fPIC", "-ffp-contract=off", "-fno-slp-vectorize", "-Wall",
         "-mllvm", "-instcombine-max-copied-from-constant-users=4000", f"--offload-arch={ARCH}"]
LIBS = ["-lz", "-lcrypto", "-lpthread", "-lrccl"]
# per-unit code generation: the hard-shadow modes (EXT 0 / 1: the C3 frames)
# schedule for instruction-level parallelism (LLVM's GCN max-ilp strategy):
# identical code semantics, C3 v1 -1.5 to -1.8 %, full quality -0.6 to -0.9 %
# (profiles/r05_ab_ilp_c3.txt, r05_ab_sched_c*.txt); the soft-shadow and
# general units keep the default occupancy-driven schedule
UNIT_FLAGS: dict[str, list[str]] = {
    "vx_render_e0.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    "vx_render_e1.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
}


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.sep not in cand or os.path.exists(cand)):
            return cand
    raise RuntimeError("hipcc not found")


CLI = os.path.join(HERE, "vxrender")


def build_cli(verbose: bool = False) -> str:
    """The C++ host (csrc/vx_cli.cpp) over the C ABI, linked to the in-tree library."""
    cmd = [hipcc(), "-O2", "-std=c++20", f"--offload-arch={ARCH}", "-o", CLI, os.path.join(CSRC, "vx_cli.cpp"),
           f"-L{HERE}", "-lvoxmap_hip", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return CLI


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [os.path.join(HERE, "..", "include", "voxmap.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = True, out: str | None = None, defines=(), extra_flags=()) -> str:
    """Build the library.  ``out``/``defines`` make experiment variants (A/B runs
    select one with VOXMAP_LIB=path); the product is always the default build."""
    target = out or OUT
    if out is None and not defines and not extra_flags and not force and not needs_build():
        return OUT
    tmp = target + ".tmp"
    # one object per source, compiled in parallel (the kernels file dominates)
    tag = os.path.basename(target).replace(".", "_")
    objdir = os.path.join(HERE, "build", tag)
    os.makedirs(objdir, exist_ok=True)
    flags = [*FLAGS, *extra_flags, *[f"-D{d}" for d in defines]]
    jobs, objs = [], []
    hdrs = [*(os.path.join(CSRC, h) for h in HEADERS), os.path.join(HERE, "..", "include", "voxmap.h"), __file__]
    for src in SOURCES:
        obj = os.path.join(objdir, src + ".o")
        objs.append(obj)
        # incremental unless forced: an object newer than its source and the headers is kept
        if not force and os.path.exists(obj) and all(os.path.getmtime(obj) > os.path.getmtime(d)
                                                     for d in [os.path.join(CSRC, src), *hdrs]):
            continue
        cmd = [hipcc(), *flags, *UNIT_FLAGS.get(src, []), "-c", "-o", obj, os.path.join(CSRC, src)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        jobs.append((cmd, obj))
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=max(1, min(len(jobs), os.cpu_count() or 1, 8))) as ex:
        for r in list(ex.map(lambda j: subprocess.run(j[0]), jobs)):
            if r.returncode:
                raise subprocess.CalledProcessError(r.returncode, r.args)
    cmd = [hipcc(), *flags, "-shared", "-o", tmp, *objs, *LIBS]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    if not defines and not extra_flags:
        # the product must keep 8 waves/SIMD and no KernelArgs scratch copy
        from . import kernel_meta
        try:
            kernel_meta.check(tmp)
        except Exception:
            os.remove(tmp)
            raise
    os.replace(tmp, target)
    if out is None:
        build_cli(verbose)
    return target


if __name__ == "__main__":
    build(force="--force" in sys.argv)
