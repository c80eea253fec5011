"""Box-Muller variants vs torch.randn on the device generator (probe for tdmpc_reference_normals)."""
import ctypes as C, os, sys
import torch
L = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "bm_probe.so"))
L.bm_probe.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_int]
n = 200000
torch.cuda.init()
gen = torch.cuda.default_generators[0]
torch.manual_seed(77)
off = gen.get_offset()
ref = torch.randn(n, device="cuda")
out = torch.empty(n, device="cuda")
for v in [-1] + list(range(16)):
    assert L.bm_probe(out.data_ptr(), n, 77, off, v) == 0
    d = (out != ref)
    ulp = (out.view(torch.int32) - ref.view(torch.int32)).abs().max().item()
    print(f"variant {v:3d}: {int(d.sum())} of {n} differ, max ulp {ulp}")
