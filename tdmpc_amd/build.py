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
        os.path.join(HERE, "csrc", "learner_conv.hip"),
        os.path.join(HERE, "csrc", "learner_kernels.hip"), os.path.join(HERE, "csrc", "learner_engine.hip")]
OUT = os.path.join(HERE, "libtdmpc_hip.so")
ARCH = os.environ.get("TDMPC_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def build(force: bool = False, verbose: bool = True, variant: str = "", defines=()) -> str:
    """The library (every source compiled in parallel, then linked); a variant (-DNAME defines, diagnostics or an A/B
    of a kernel knob) goes to libtdmpc_hip_<variant>.so, loaded with TDMPC_LIB_PATH."""
    deps = SRCS + [os.path.join(HERE, "csrc", f) for f in ("plan1.inc", "wide_step.inc", "wide_heads.inc")] + \
        [os.path.join(REPO, "include", h) for h in ("tdmpc_hip.h", "tdmpc_replay.h", "tdmpc_learner.h")]
    out = OUT if not variant else os.path.join(HERE, f"libtdmpc_hip_{variant}.so")
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    # -fno-slp-vectorize: no packed v_pk_add/mul_f32 from pairs of scalar f32 ops -- beside MFMAs a packed f32 VALU
    # instruction costs ~+22-26 cycles where two scalar ones are free (MI355X_MICROARCH.md, filler prices)
    base = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize",
            "-I", os.path.join(REPO, "include")] + [f"-D{d}" for d in defines] + \
        ([f"-DTDMPC_VARIANT={variant}"] if variant else [])
    objs, procs = [], []
    for src in SRCS:
        obj = os.path.join(HERE, "csrc", os.path.basename(src) + (f".{variant}" if variant else "") + ".o")
        cmd = base + ["-c", "-o", obj, src]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    if any(p.wait() != 0 for p in procs):
        raise subprocess.CalledProcessError(1, "hipcc")
    tmp = out + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    for o in objs:
        os.remove(o)
    os.replace(tmp, out)
    return out


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
    # python -m tdmpc_amd.build [--force] [--variant NAME -DDEFINE ...]
    args = sys.argv[1:]
    var = args[args.index("--variant") + 1] if "--variant" in args else ""
    defs = [a[2:] for a in args if a.startswith("-D")]
    build(force="--force" in args or bool(var), variant=var, defines=defs)
    if not var:
        build_example(force="--force" in args)
