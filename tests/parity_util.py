"""Shared parity helpers for the GPU tests (tolerances: see tests/test_gpu_plan.py's header).

Near-tie accounting: a plan whose elite set differs from the oracle's only by candidates within 1e-4
(relative) of the cut-off value diverges legitimately from then on, and its later iterations / calls are not
compared. Every such escape is counted here instead of being skipped silently;
tests/test_zz_parity_budget.py requires that at least 90 % of the plan comparisons of the session ran to the
end (action, mean, std and metrics compared)."""
import numpy as np

RTOL, ATOL = 1e-4, 1e-5

TIES = {"full": 0, "escaped": 0, "where": []}


def record(full: bool, where: str = ""):
    if full:
        TIES["full"] += 1
    else:
        TIES["escaped"] += 1
        TIES["where"].append(where)


def close(a, b, atol=ATOL, rtol=RTOL):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.abs(a - b) <= atol + rtol * np.abs(b)


def elites(v, K):
    return set(np.argsort(-np.asarray(v), kind="stable")[:K].tolist())


def near_tie(ref_v, a, b, K):
    """True when the symmetric difference of two elite sets only holds values next to the cut-off."""
    v = np.asarray(ref_v, dtype=np.float64)
    cut = np.sort(v)[::-1][K - 1]
    diff = a ^ b
    return all(abs(v[i] - cut) <= 1e-4 * (1 + abs(cut)) for i in diff)


def compare_iterations(gpu_vals, ref_vals, K):
    """Compare per-iteration values; returns True if every iteration's elite set agreed (False: a near-tie
    swap, after which the iterations diverge legitimately; anything else fails)."""
    for i in range(ref_vals.shape[0]):
        ok = close(gpu_vals[i], ref_vals[i])
        assert ok.all(), f"iteration {i}: max |dG| {np.abs(gpu_vals[i] - ref_vals[i]).max():.3e}"
        eg, er = elites(gpu_vals[i], K), elites(ref_vals[i], K)
        if eg != er:
            assert near_tie(ref_vals[i], eg, er, K), f"iteration {i}: elite sets differ away from the cut-off"
            return False
    return True
