"""One GEMM shape through ds2_sgemm_ws for a profiler (rocprofv3 --pmc / --kernel-trace).
usage: python scripts/gemm_one.py TA TB M N K [iters]   (DS2_GEMM_X6 selects the kernel)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
from ds2amd import ops  # noqa: E402

ta, tb, m, n, k = (int(v) for v in sys.argv[1:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 5
dev = torch.device("cuda")
a = torch.randn((k, m) if ta else (m, k), device=dev)
b = torch.randn((n, k) if tb else (k, n), device=dev)
c = torch.empty(m, n, device=dev)
for _ in range(iters):
    ops.sgemm(a, b, c, m=m, n=n, k=k, trans_a=bool(ta), trans_b=bool(tb), lda=a.shape[1],
              ldb=b.shape[1], ldc=n)
torch.cuda.synchronize()
print("ok", ta, tb, m, n, k, os.environ.get("DS2_GEMM_X6", "1"))
