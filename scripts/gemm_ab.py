"""A/B: TN GEMM via the LDS-DMA kernel vs the register-staged kernel (same process)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch
from ds2amd import ops
dev = torch.device("cuda")
def timeit(fn, iters=20):
    fn(); torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / iters
for (m, n, k) in [(2400, 800, 16032), (2400, 1312, 16032), (4096, 4096, 4096), (2400, 800, 15999)]:
    A = torch.randn(k, m, device=dev); B = torch.randn(k, n, device=dev); C = torch.empty(m, n, device=dev)
    f = lambda: ops.sgemm(A, B, C, m=m, n=n, k=k, trans_a=True, lda=m, ldb=n, ldc=n)
    res = {}
    for flag in ("1", "0"):
        os.environ["DS2_GEMM_TN_DMA"] = flag
        res[flag] = timeit(f)
        out = C.clone()
        res[flag + "o"] = out
    fl = 2.0 * m * n * k
    diff = (res["1o"] - res["0o"]).abs().max().item() / res["0o"].abs().max().item()
    print(f"TN {m}x{n}x{k}: dma {res['1']*1e3:.0f} us {fl/res['1']/1e9:.1f} TF | reg {res['0']*1e3:.0f} us {fl/res['0']/1e9:.1f} TF | rel diff {diff:.2e}")
