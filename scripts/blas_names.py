"""Run hipBLASLt fp32 GEMMs on the model's shapes once each (for rocprofv3 kernel names)."""
import torch

dev = torch.device("cuda")
for ta, tb, m, n, k in [(0, 1, 16032, 2400, 800), (0, 0, 16032, 1312, 2400),
                        (1, 0, 2400, 800, 16032), (0, 0, 4096, 4096, 4096)]:
    a = torch.randn((k, m) if ta else (m, k), device=dev)
    b = torch.randn((n, k) if tb else (k, n), device=dev)
    at = a.t() if ta else a
    bt = b.t() if tb else b
    for _ in range(3):
        torch.mm(at, bt)
    torch.cuda.synchronize()
