"""Microbenchmark: ds2_sgemm_ws on the model's GEMM shapes vs torch (rocBLAS/hipBLASLt) fp32."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
from ds2amd import ops  # noqa: E402

dev = torch.device("cuda")
torch.backends.cuda.matmul.allow_tf32 = False
SHAPES = [  # name, ta, tb, m, n, k
    ("xproj NT", 0, 1, 16032, 2400, 1312),
    ("xproj NT", 0, 1, 16032, 2400, 800),
    ("dX NN", 0, 0, 16032, 800, 2400),
    ("dX NN", 0, 0, 16032, 1312, 2400),
    ("dW TN", 1, 0, 2400, 800, 16032),
    ("dW TN", 1, 0, 2400, 1312, 16032),
    ("sq NN", 0, 0, 4096, 4096, 4096),
]


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s0 = torch.cuda.Event(enable_timing=True); s1 = torch.cuda.Event(enable_timing=True)
    s0.record()
    for _ in range(iters):
        fn()
    s1.record()
    torch.cuda.synchronize()
    return s0.elapsed_time(s1) / iters


for name, ta, tb, m, n, k in SHAPES:
    a = torch.randn((k, m) if ta else (m, k), device=dev)
    b = torch.randn((n, k) if tb else (k, n), device=dev)
    c = torch.empty(m, n, device=dev)
    f1 = lambda: ops.sgemm(a, b, c, m=m, n=n, k=k, trans_a=bool(ta), trans_b=bool(tb),
                           lda=a.shape[1], ldb=b.shape[1], ldc=n)
    at = a.t() if ta else a
    bt = b.t() if tb else b
    f2 = lambda: torch.mm(at, bt, out=c)
    fl = 2.0 * m * n * k
    os.environ["DS2_GEMM64"] = "0"
    t0 = timeit(f1)
    r0 = c.clone()
    os.environ["DS2_GEMM64"] = "1"
    res = []
    for bn in ("128", "160"):
        os.environ["DS2_GEMM_BN"] = bn
        t1 = timeit(f1)
        rel = ((c - r0).abs().max() / r0.abs().max()).item()
        res.append(f"bk64/{bn} {fl/t1/1e9:6.1f} TF ({rel:.0e})")
    del os.environ["DS2_GEMM_BN"]
    t1 = timeit(f1)
    t2 = timeit(f2)
    print(f"{name:9s} {m:6d}x{n:5d}x{k:6d}: bk16 {fl/t0/1e9:6.1f} | " + " | ".join(res) +
          f" | auto {t1*1e3:7.1f} us {fl/t1/1e9:6.1f} | torch {fl/t2/1e9:6.1f} TF", flush=True)
