"""Build libcwt.so in-tree with hipcc for gfx950 (no torch extension machinery needed:
the library is a plain C ABI loaded through ctypes).

    python -m few_shot_seg_cwt_amd.build [--force]
"""
from __future__ import annotations

import hashlib
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "csrc", "build")
LIB = os.path.join(HERE, "libcwt.so")
SOURCES = ["api.hip", "conv.hip", "conv_x3s.hip", "backbone.hip", "adapt.hip", "cwt_attn.hip", "seg.hip",
           "bn_train.hip", "preprocess.hip", "heads.hip", "match.hip", "detr.hip", "pretrain_kernels.hip",
           "pretrain.hip", "tail.hip", "match_bwd.hip", "wino.hip", "conv_x6.hip"]
HEADERS = ["common.h", "kernels.h", "pretrain.h", "conv_plans_x3s.inc", "conv_plans_b16.inc", "conv_plans_f32.inc", "conv_plans_f32d.inc", "conv_plans_x6.inc", "conv_body.h", "tail_body.h"]
PUBLIC_HEADERS = ["cwt.h", "cwt_debug.h"]
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-munsafe-fp-atomics"]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


def _deps():
    return ([os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(INCLUDE, f) for f in PUBLIC_HEADERS])


def source_hash() -> str:
    """Content hash (16 hex digits) of every HIP source and header the library is built from.
    It is compiled into cwt_version() ("src=<hash>") and checked against the tree when the
    library is loaded (_lib.load_library), so a stale binary is refused, never run."""
    h = hashlib.sha256()
    for p in _deps():
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def built_hash(path: str = LIB):
    """The source hash compiled into a built library (None if absent or unmarked)."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        m = re.search(rb"libcwt [0-9.]+ \(gfx950\) src=([0-9a-f]{16})", f.read())
    return m.group(1).decode() if m else None


def _compile(src: str, force: bool, src_hash: str) -> str:
    s = os.path.join(CSRC, src)
    o = os.path.join(OBJ, src.replace(".hip", ".o"))
    stamp = o + ".hash"
    own = [s] + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INCLUDE, h) for h in PUBLIC_HEADERS]
    if not force and _mtime(o) >= max(_mtime(d) for d in own) and \
            (src != "api.hip" or (os.path.exists(stamp) and open(stamp).read() == src_hash)):
        return o
    extra = [f'-DCWT_SRC_HASH="{src_hash}"'] if src == "api.hip" else []
    cmd = [HIPCC, *FLAGS, *extra, "-c", s, "-o", o]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    if src == "api.hip":
        with open(stamp, "w") as f:
            f.write(src_hash)
    return o


def build(force: bool = False, verbose: bool = True) -> str:
    """Up to date iff the library's compiled-in source hash equals the tree's (content, not
    mtimes: the GPU box receives the library without the object files)."""
    src_hash = source_hash()
    if not force and built_hash() == src_hash:
        if verbose:
            print(f"up to date: {LIB} (src={src_hash})")
        return LIB
    os.makedirs(OBJ, exist_ok=True)
    with ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, src_hash), SOURCES))
    # -z defs: an undefined symbol fails the link instead of the first dlopen
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-Wl,-z,defs", "-o", LIB, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if built_hash() != src_hash:
        raise RuntimeError(f"built {LIB} but its source hash is {built_hash()}, expected {src_hash}")
    if verbose:
        print(f"built {LIB} (src={src_hash})")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
