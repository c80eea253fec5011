"""Pin the oracle: the CPU restatement must reproduce the reference's own outputs (golden vectors generated
by running /root/reference's TDMPC.plan in the build container, tests/golden/make_golden.py) bit-exactly."""
import numpy as np
import pytest
import torch

from oracle import tdmpc_ref
from tdmpc_amd.told import synthetic_state_dict
from golden_io import case_names, load_case, call_noise


@pytest.fixture
def one_thread():
    """The plan fixtures were recorded at one intra-op thread; restored after, because other fixtures (the learner's)
    were recorded at the container's default and their CPU reductions depend on the thread count."""
    n = torch.get_num_threads()
    torch.set_num_threads(1)
    yield
    torch.set_num_threads(n)


@pytest.mark.parametrize("name", case_names())
def test_oracle_matches_reference_golden(name, one_thread):
    cfg, wseed, d = load_case(name)
    sd = synthetic_state_dict(cfg, wseed)
    fp = np.array([float(v.double().sum()) for v in sd.values()])
    np.testing.assert_array_equal(fp, d["w_fingerprint"])
    told = tdmpc_ref.RefTOLD(sd, cfg)
    state = tdmpc_ref.PlanState(0.05)
    for ci in range(int(d["ncalls"])):
        step, t0, ev = [int(x) for x in d[f"c{ci}_call"]]
        trace = {}
        a, m = tdmpc_ref.plan(told, cfg, state, d[f"c{ci}_obs"], call_noise(d, ci), eval_mode=bool(ev),
                              step=step, t0=bool(t0), trace=trace)
        np.testing.assert_array_equal(a.numpy(), d[f"c{ci}_action"])
        assert [m["external_reward_mean"], m["current_std"]] == list(d[f"c{ci}_metrics"])
        if f"c{ci}_values" in d:
            np.testing.assert_array_equal(torch.stack(trace["value"]).squeeze(-1).numpy(), d[f"c{ci}_values"])
            np.testing.assert_array_equal(np.array(trace["reward_mean"]), d[f"c{ci}_reward_means"])
        if f"c{ci}_prev_mean" in d and state.prev_mean is not None:
            np.testing.assert_array_equal(state.prev_mean.numpy(), d[f"c{ci}_prev_mean"])


def test_choice_index_matches_numpy():
    rs = np.random.RandomState(0)
    for _ in range(200):
        p = rs.random_sample(64).astype(np.float32)
        p /= p.sum()
        st = np.random.RandomState(rs.randint(1 << 30))
        st2 = np.random.RandomState(0); st2.set_state(st.get_state())
        j = st.choice(np.arange(64), p=p)
        assert tdmpc_ref.choice_index(p, st2.random_sample()) == j
