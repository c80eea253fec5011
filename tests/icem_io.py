"""Shared by tests/golden/make_icem_golden.py and tests/test_icem.py: the iCEM golden case."""
from tdmpc_amd.config import make_cfg

# (step, t0, eval_mode): horizon schedule linear(2, 5, 25000) gives H = 3 at step 10000, 4 at 17000, 5 at 1e6;
# regularization_schedule (humanoid) linear(0.05, 0.5, 1, 50000) gives mixture 0.05 / 0.05 / 0.5
CALLS = [(10000, True, False), (10000, False, False), (17000, True, False), (17000, False, True),
         (10**6, True, False), (10**6, False, False)]


def icem_cfg():
    """humanoid dims (latent 100, LayerNorm state encoder), N = 64 shrinking by 1.25, 8 elites (2 reused),
    3 iterations, the reference's iCEM defaults (cfgs/default.yaml:17-24)."""
    return make_cfg("humanoid", num_samples=64, num_elites=8, iterations=3, horizon=5)
