"""Build libnrk.so (HIP, gfx950) and the oracle's C library, in-tree.

    python -m newsrecommend_amd.build            # both
The product library goes to newsrecommend_amd/libnrk.so; the test-only oracle
library to oracle/liboracle_knn.so.  Both are git-ignored build outputs that
travel to the GPU box with the working tree.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libnrk.so")
ORACLE_SRC = os.path.join(ROOT, "oracle", "knn_exact.c")
ORACLE_LIB = os.path.join(ROOT, "oracle", "liboracle_knn.so")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"]
SOURCES = ["nrk_common.cpp", "click_log.cpp", "knn_flat.hip", "din_attn.hip", "ivf_build.hip", "din_head.hip", "din_rerank.hip", "din_rerank_lane.hip", "embed.hip",
           "screen_dp32.hip", "screen_dp64.hip", "screen_dp128.hip", "screen_dp256.hip"]
# din_rerank: no NaN inputs (finite weights and table rows; padded candidates are
# written as -inf, never computed), so max / min need no IEEE canonicalisation
FILE_FLAGS = {"din_rerank.hip": ["-fno-honor-nans", "-mno-amdgpu-ieee"],
              "din_rerank_lane.hip": ["-fno-honor-nans", "-mno-amdgpu-ieee", "-fno-slp-vectorize"]}


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def _newer(target, deps):
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def build_lib(force: bool = False) -> str:
    headers = [os.path.join(CSRC, "nrk_common.h"), os.path.join(CSRC, "din_rerank.h"), os.path.join(CSRC, "screen.h"), os.path.join(CSRC, "screen16.h"), os.path.join(ROOT, "include", "nrk.h")]
    objdir = os.path.join(CSRC, "build")
    os.makedirs(objdir, exist_ok=True)
    jobs = []
    objs = []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(objdir, os.path.splitext(s)[0] + ".o")
        objs.append(obj)
        if force or not _newer(obj, [src, *headers]):
            lang = ["-x", "hip"] if s.endswith(".hip") else []
            jobs.append([HIPCC, *HIP_FLAGS, *FILE_FLAGS.get(s, []), *lang, "-c", src, "-o", obj])
    with cf.ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        list(ex.map(_run, jobs))
    if jobs or not _newer(LIB, objs):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", LIB])
    return LIB


def build_oracle(force: bool = False) -> str:
    if force or not _newer(ORACLE_LIB, [ORACLE_SRC]):
        _run(["gcc", "-O2", "-fopenmp", "-shared", "-fPIC", "-std=c11", ORACLE_SRC, "-o", ORACLE_LIB, "-lm"])
    return ORACLE_LIB


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    force = "--force" in argv
    print(build_lib(force))
    print(build_oracle(force))


if __name__ == "__main__":
    main()
