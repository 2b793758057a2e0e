"""Probe: fp32 GEMM rate of rocBLAS and hipBLASLt (through torch.mm) vs ds2_sgemm_ws on the
model's shapes, and whether repeated library calls are bitwise reproducible."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
from ds2amd import ops  # noqa: E402

dev = torch.device("cuda")
SHAPES = [("xproj NT", 0, 1, 16032, 2400, 1312), ("xproj NT", 0, 1, 16032, 2400, 800),
          ("dX NN", 0, 0, 16032, 800, 2400), ("dX NN", 0, 0, 16032, 1312, 2400),
          ("dW TN", 1, 0, 2400, 800, 16032), ("dW TN", 1, 0, 2400, 1312, 16032),
          ("sq NN", 0, 0, 4096, 4096, 4096)]


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s0 = torch.cuda.Event(enable_timing=True)
    s1 = torch.cuda.Event(enable_timing=True)
    s0.record()
    for _ in range(iters):
        fn()
    s1.record()
    torch.cuda.synchronize()
    return s0.elapsed_time(s1) / iters


print("default preferred blas:", torch.backends.cuda.preferred_blas_library(), flush=True)
for name, ta, tb, m, n, k in SHAPES:
    a = torch.randn((k, m) if ta else (m, k), device=dev)
    b = torch.randn((n, k) if tb else (k, n), device=dev)
    c = torch.empty(m, n, device=dev)
    at = a.t() if ta else a
    bt = b.t() if tb else b
    fl = 2.0 * m * n * k
    f1 = lambda: ops.sgemm(a, b, c, m=m, n=n, k=k, trans_a=bool(ta), trans_b=bool(tb),
                           lda=a.shape[1], ldb=b.shape[1], ldc=n)
    res = [f"ds2 {fl / timeit(f1) / 1e9:6.1f}"]
    for lib in ("cublas", "cublaslt"):
        torch.backends.cuda.preferred_blas_library(lib)
        f2 = lambda: torch.mm(at, bt, out=c)
        t = timeit(f2)
        r1 = torch.mm(at, bt)
        r2 = torch.mm(at, bt)
        same = torch.equal(r1, r2)
        res.append(f"{lib} {fl / t / 1e9:6.1f} (repro {same})")
    torch.backends.cuda.preferred_blas_library("default")
    print(f"{name:9s} {m:6d}x{n:5d}x{k:6d} TF: " + " | ".join(res), flush=True)
