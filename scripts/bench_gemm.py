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
    variants = [("bk16", {"DS2_GEMM64": "0"}), ("sb128", {"DS2_GEMM_BN": "128"}),
                ("sb160", {"DS2_GEMM_BN": "160"}), ("db128", {"DS2_GEMM_BN": "128", "DS2_GEMM_DB": "1"}),
                ("db160", {"DS2_GEMM_BN": "160", "DS2_GEMM_DB": "1"})]
    res, ref = [], None
    for vname, env in variants:
        for key in ("DS2_GEMM64", "DS2_GEMM_BN", "DS2_GEMM_DB"):
            os.environ.pop(key, None)
        os.environ.update(env)
        t1 = timeit(f1)
        if ref is None:
            ref = c.clone()
        rel = ((c - ref).abs().max() / ref.abs().max()).item()
        res.append(f"{vname} {fl/t1/1e9:6.1f}" + ("" if rel < 1e-5 else f" (rel {rel:.0e}!)"))
    for key in ("DS2_GEMM64", "DS2_GEMM_BN", "DS2_GEMM_DB"):
        os.environ.pop(key, None)
    t2 = timeit(f2)
    print(f"{name:9s} {m:6d}x{n:5d}x{k:6d} TF: " + " | ".join(res) + f" | torch {fl/t2/1e9:6.1f}",
          flush=True)
