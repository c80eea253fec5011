import torch
dev = torch.device("cuda")
for (m, n, k) in [(2560, 512, 512), (3072, 512, 512), (512, 512, 512), (16384, 512, 512), (2560, 512, 2560)]:
    a = torch.randn(m, k, device=dev); b = torch.randn(n, k, device=dev)
    for _ in range(5): c = a @ b.t()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50): c = a @ b.t()
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 50
    print(f"torch.mm fp32 {m}x{n}x{k}: {us:.1f} us {2*m*n*k/us/1e6:.1f} TFLOP/s", flush=True)
