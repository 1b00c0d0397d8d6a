"""Build libcwt.so in-tree with hipcc for gfx950 (no torch extension machinery needed:
the library is a plain C ABI loaded through ctypes).

    python -m few_shot_seg_cwt_amd.build [--force]
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "csrc", "build")
LIB = os.path.join(HERE, "libcwt.so")
SOURCES = ["api.hip", "conv.hip", "conv_x3.hip", "conv_x3s.hip", "backbone.hip", "adapt.hip", "cwt_attn.hip", "seg.hip",
           "bn_train.hip", "preprocess.hip"]
HEADERS = ["common.h", "kernels.h", "conv_plans.inc", "conv_plans_x3s.inc", "conv_plans_b16.inc"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-munsafe-fp-atomics"]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


def _compile(src: str, force: bool) -> str:
    s = os.path.join(CSRC, src)
    o = os.path.join(OBJ, src.replace(".hip", ".o"))
    deps = [s] + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(os.path.dirname(HERE), "include", "cwt.h")]
    if not force and _mtime(o) >= max(_mtime(d) for d in deps):
        return o
    cmd = [HIPCC, *FLAGS, "-c", s, "-o", o]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return o


def build(force: bool = False, verbose: bool = True) -> str:
    srcs = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(os.path.dirname(HERE), "include", "cwt.h")]
    if not force and _mtime(LIB) >= max(_mtime(p) for p in srcs):
        # up to date (the GPU box gets the library but not the object files)
        if verbose:
            print(f"up to date: {LIB}")
        return LIB
    os.makedirs(OBJ, exist_ok=True)
    with ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), SOURCES))
    if force or _mtime(LIB) < max(_mtime(o) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
