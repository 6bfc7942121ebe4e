"""Builds the in-tree native library ``libptgpu.so`` for gfx950 with hipcc.

The library holds the HIP kernels (csrc/pt_kernels.hip), the C ABI
(csrc/pt_api.cpp, include/ptgpu.h) and the native host scene pipeline
(csrc/scene_host.cpp).  It is built in-tree so that it travels with the
repository snapshot to the GPU box; nothing is installed.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libptgpu.so")
ARCH = os.environ.get("PT_OFFLOAD_ARCH", "gfx950")


def _sources():
    return [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith((".hip", ".cpp"))]


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    inc = os.path.join(ROOT, "include")
    hs += [os.path.join(inc, f) for f in os.listdir(inc) if f.endswith(".h")]
    return hs


def up_to_date() -> bool:
    if os.environ.get("PT_HIPCC_FLAGS") or os.environ.get("PT_KERNEL_SCHED") or os.environ.get("PT_ENV_SCHED"):
        return False
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    if not os.path.exists(SEAM_BENCH):
        return False
    return all(os.path.getmtime(p) <= t for p in _sources() + _headers() + [__file__])


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP path cannot be built")


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    objdir = os.path.join(PKG, "_obj")
    os.makedirs(objdir, exist_ok=True)
    objs = []
    procs = []
    for src in _sources():
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
               "-Wno-unused-function", f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}", "-c", src, "-o", obj]
        cmd[1:1] = os.environ.get("PT_HIPCC_FLAGS", "").split()  # experiments, e.g. -DPT_MIN_WAVES_PER_SIMD=5
        base = os.path.basename(src)
        if base in ("pt_kernels.hip", "pt_kernels_env.hip"):
            # SLP-packed float3 math (v_pk_*_f32) needs operand shuffles that
            # cost more VALU slots and VGPRs than the pairing saves here
            # (render_kernel 103 -> 99 VGPRs; C3 +3.5%)
            cmd.insert(1, "-fno-slp-vectorize")
        # machine scheduler per kernel translation unit (experiments: "default"
        # drops the flag, any other value is passed as the strategy name)
        sched = os.environ.get("PT_KERNEL_SCHED", "max-ilp")
        env_sched = os.environ.get("PT_ENV_SCHED", "iterative-ilp")
        strategy = {"pt_kernels.hip": sched, "pt_kernels_env.hip": env_sched}.get(base, "default")
        if strategy == "ilp":
            strategy = "iterative-ilp"
        if strategy != "default":
            # common build: iterative-ILP scheduling measured C3 +1.7% in round 2,
            # max-ILP +1.0-1.5% over it in round 4 (profiles/r4/ab_sched_strategy.txt,
            # ab_env_uv_groups.txt); the ENV build stays iterative-ILP (C5 +0.8%
            # with the round-3 follow-up rays; max-ILP neutral)
            cmd[1:1] = ["-mllvm", f"-amdgpu-sched-strategy={strategy}"]
        if src.endswith(".cpp") and "pt_api" not in src:
            cmd.insert(1, "-xc++")  # host-only translation units
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        objs.append(obj)
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"build failed: {' '.join(cmd)}\n{out.decode(errors='replace')}")
        if verbose and out:
            sys.stderr.write(out.decode(errors="replace"))
    tmp = LIB + ".tmp"
    link = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + ["-lz"]
    r = subprocess.run(link, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(link)}\n{r.stdout.decode(errors='replace')}")
    os.replace(tmp, LIB)
    build_seam_bench()
    return LIB


SEAM_BENCH = os.path.join(PKG, "seam_bench")


def build_seam_bench() -> str:
    """tools/seam_bench.cpp: the C++ driver of the per-tile seam (bench.py's
    c3_per_tile companions), linked against the in-tree libptgpu.so."""
    src = os.path.join(ROOT, "tools", "seam_bench.cpp")
    cmd = ["g++", "-O2", "-std=c++17", "-pthread", f"-I{os.path.join(ROOT, 'include')}", src, "-o", SEAM_BENCH,
           f"-L{PKG}", "-lptgpu", "-Wl,-rpath,$ORIGIN"]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError(f"seam_bench build failed: {' '.join(cmd)}\n{r.stdout.decode(errors='replace')}")
    return SEAM_BENCH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
