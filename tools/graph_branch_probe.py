"""When does the second branch of a captured HIP graph start? (development tool)
    python tools/graph_branch_probe.py
Branch A: a chain of NA short kernels (tdmpc_lg_act over 1 M floats) on the capturing stream; branch B: ONE long kernel
(tdmpc_lg_act over 64 M floats) on a second stream forked from it. Graph replay times (HIP events, median of 20):
A alone, B alone, and A + B captured with A's launches first, B's first, or interleaved. Concurrent branches give
max(A, B); a branch whose start waits for the other branch's launches to be dispatched gives about their sum."""
import ctypes as C
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from tdmpc_amd import _lib

lib = _lib.lib()
dev = torch.device("cuda")
NA = int(os.environ.get("NA", "25"))
xs = torch.zeros(1 << 20, device=dev)
xl = torch.zeros(64 << 20, device=dev)


def act(x):
    rc = lib.tdmpc_lg_act(x.data_ptr(), None, x.numel(), 0, C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0


def build(order):
    g = torch.cuda.CUDAGraph()
    main = torch.cuda.Stream()
    side = torch.cuda.Stream()
    a = [lambda: act(xs)] * NA if order != "b" else []
    b = [lambda: act(xl)] if order != "a" else []
    with torch.cuda.graph(g, stream=main):
        side.wait_stream(main)
        seq = {"a": [(main, f) for f in a], "b": [(side, f) for f in b],
               "ab": [(main, f) for f in a] + [(side, f) for f in b],
               "ba": [(side, f) for f in b] + [(main, f) for f in a],
               "int": ([(main, a[0]), (side, b[0])] + [(main, f) for f in a[1:]]) if a and b else []}[order]
        for st, f in seq:
            with torch.cuda.stream(st):
                f()
        main.wait_stream(side)
    return g


def time_graph(g, reps=20):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts)


for order in ("a", "b", "ab", "ba", "int"):
    g = build(order)
    g.replay()
    torch.cuda.synchronize()
    print(f"NA={NA} order {order:>3}: {time_graph(g):8.1f} us per replay", flush=True)
