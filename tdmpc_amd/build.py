"""Build libtdmpc_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m tdmpc_amd.build           # -> tdmpc_amd/libtdmpc_hip.so
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, "csrc", "tdmpc_kernels.hip"), os.path.join(HERE, "csrc", "replay_kernels.hip"),
        os.path.join(HERE, "csrc", "learner_kernels.hip"), os.path.join(HERE, "csrc", "learner_engine.hip")]
OUT = os.path.join(HERE, "libtdmpc_hip.so")
ARCH = os.environ.get("TDMPC_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def build(force: bool = False, verbose: bool = True) -> str:
    deps = SRCS + [os.path.join(HERE, "csrc", "plan1.inc"), os.path.join(HERE, "csrc", "wide_step.inc")] + [os.path.join(REPO, "include", h) for h in ("tdmpc_hip.h", "tdmpc_replay.h", "tdmpc_learner.h")]
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        return OUT
    tmp = OUT + ".tmp"
    # -fno-slp-vectorize: no packed v_pk_add/mul_f32 from pairs of scalar f32 ops -- beside MFMAs a packed f32 VALU
    # instruction costs ~+22-26 cycles where two scalar ones are free (MI355X_MICROARCH.md, filler prices)
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-fno-slp-vectorize",
           "-I", os.path.join(REPO, "include"), "-o", tmp] + SRCS
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    return OUT


EXAMPLE_SRC = os.path.join(REPO, "examples", "plan_c.cpp")
EXAMPLE_OUT = os.path.join(REPO, "examples", "plan_c")


def build_example(force: bool = False, verbose: bool = True) -> str:
    """examples/plan_c: a plain C++ host of the C ABI, linked against the in-tree library (rpath $ORIGIN)."""
    deps = [EXAMPLE_SRC, OUT, os.path.join(REPO, "include", "tdmpc_hip.h")]
    if not force and os.path.exists(EXAMPLE_OUT) and all(os.path.getmtime(EXAMPLE_OUT) >= os.path.getmtime(d)
                                                          for d in deps):
        return EXAMPLE_OUT
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O2", "-std=c++17", "-o", EXAMPLE_OUT + ".tmp", EXAMPLE_SRC,
           "-L", HERE, "-ltdmpc_hip", "-Wl,-rpath,$ORIGIN/../tdmpc_amd"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(EXAMPLE_OUT + ".tmp", EXAMPLE_OUT)
    return EXAMPLE_OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    build_example(force="--force" in sys.argv)
