"""GPU: the packed buffer's job-table nonce (include/tdmpc_hip.h, TDMPC_STATUS_PACK_STALE).

tdmpc_pack_weights keeps its job table in the caller's packed buffer. A pack captured into a HIP graph uploads
nothing and reads whatever table the buffer holds when it runs, so the library names every uploaded table by a
nonce in the buffer's header and each pack launch checks it on the device. These tests drive the two ways a pack
could otherwise read a table it was not issued for -- and pack zeros or another model's tensors with status 0:
  * a planner's buffer freed and re-allocated at the same address (zero-filled, no tdmpc_pack_forget), then packed
    first under a stream capture through the raw ABI;
  * a graph captured over a pack, after which the buffer is packed (uncaptured) from OTHER tensors.
Both must end in a raised status (NaN weights, NaN actions), never in a silent result.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from tdmpc_amd import _lib
from tdmpc_amd.config import make_cfg
from tdmpc_amd.tdmpc import TDMPC
from tdmpc_amd.told import synthetic_state_dict

pytestmark = pytest.mark.gpu


def _agent(path):
    cfg = make_cfg("humanoid", num_samples=512, num_elites=64, iterations=6, horizon=5)
    agent = TDMPC(cfg, max_batch=1, path=path)
    agent.model.load_state_dict(synthetic_state_dict(cfg, 3))
    agent.std = 0.05
    obs = np.random.RandomState(1).standard_normal(cfg.obs_shape).astype(np.float32)
    return cfg, agent, obs


def _pack_raw(pl, arr, n, stream):
    """tdmpc_pack_weights through the raw C ABI (pointer array, packed buffer, stream): returns its code."""
    return pl.L.tdmpc_pack_weights(C.byref(pl.dims), arr, n, C.c_void_p(pl.packed.data_ptr()), pl.packed.numel() * 4,
                                   C.c_void_p(stream))


def _capture_pack(pl, arr, n):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.graph(g, stream=s):
        _lib.check(_pack_raw(pl, arr, n, torch.cuda.current_stream().cuda_stream), "captured pack")
    return g


@pytest.mark.parametrize("path", ["auto", "chain_x6"])   # auto at one env: the persistent plan1 kernel
def test_stale_pack_at_reused_address_raises(path):
    cfg, agent, obs = _agent(path)
    a0, _ = agent.plan(obs, step=10**6, t0=True)   # uncaptured pack: the buffer's table + record
    assert torch.isfinite(a0).all()
    pl = agent.planner
    arr, n = pl._ptr_arr
    # free the packed buffer and allocate a zero-filled one at the same address, without tdmpc_pack_forget
    numel, p0 = pl.packed.numel(), pl.packed.data_ptr()
    pl.packed = None
    torch.cuda.synchronize()
    pl.packed = torch.zeros(numel, dtype=torch.float32, device=pl.device)
    assert pl.packed.data_ptr() == p0, "the caching allocator did not hand back the freed block"
    # the first pack into it runs under capture: the host record matches (same address, same tensors), the device
    # header does not (zeros)
    g = _capture_pack(pl, arr, n)
    g.replay()
    torch.cuda.synchronize()
    head = pl.packed[:4096]
    assert torch.isnan(head).all(), "a stale pack must poison the weights, not leave zeros"
    with pytest.raises(RuntimeError, match="job table"):
        agent.plan(obs, step=10**6, t0=True)
    assert int(pl.status.item()) == 0   # raise_status cleared the word
    # recovery: an uncaptured pack uploads the table again and clears the buffer's sticky status
    pl._packed_key = None
    a1, m1 = agent.plan(obs, step=10**6, t0=True)
    assert torch.isfinite(a1).all() and np.isfinite(list(m1.values())).all()


def test_captured_pack_refuses_other_tensors_then_stale_replay_raises():
    cfg, agent, obs = _agent("chain_x6")
    agent.plan(obs, step=10**6, t0=True)
    pl = agent.planner
    arr, n = pl._ptr_arr
    g = _capture_pack(pl, arr, n)
    g.replay()
    a0, _ = agent.plan(obs, step=10**6, t0=True)
    assert torch.isfinite(a0).all()   # a valid captured pack replays fine
    # an uncaptured pack from other tensors (a copy of the model) would re-point the captured graph: refused
    copies = [p.detach().clone() for p in agent.model.state_dict().values()]
    arr2 = (C.c_void_p * n)(*[p.data_ptr() for p in copies])
    stream = torch.cuda.current_stream().cuda_stream
    with pytest.raises(RuntimeError, match="captured graph"):
        _lib.check(_pack_raw(pl, arr2, n, stream), "re-keying pack")
    # tdmpc_pack_forget re-keys the buffer explicitly: the new pack is accepted and plans ...
    pl.L.tdmpc_pack_forget(C.c_void_p(pl.packed.data_ptr()))
    _lib.check(_pack_raw(pl, arr2, n, stream), "pack after forget")
    a1, _ = agent.plan(obs, step=10**6, t0=True)
    assert torch.isfinite(a1).all()
    # ... and the old graph's pack, replayed now, finds another table: it fails loudly at the next plan
    g.replay()
    with pytest.raises(RuntimeError, match="job table"):
        agent.plan(obs, step=10**6, t0=True)
    torch.cuda.synchronize()
    del copies
