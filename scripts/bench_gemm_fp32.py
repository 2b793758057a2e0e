"""Microbenchmark: ds2_sgemm_ws (fp32 MFMA) on the headline step's GEMM shapes (5 x BiGRU-800,
batch 32, T' = 501: TN = 16032 rows) vs torch.mm fp32 (hipBLASLt / rocBLAS) on the same
operands.  Prints TFLOP/s and the fraction of the dense fp32 MFMA peak (157.3 TFLOP/s).

usage: python scripts/bench_gemm_fp32.py [variant ...]   variant = BN:DB, e.g. 160:0 128:1
(DS2_GEMM_BN / DS2_GEMM_DB, read by the library at every call; default: the planner's choice)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
from ds2amd import ops  # noqa: E402

dev = torch.device("cuda")
TN = 501 * 32
PEAK = 157.3
SHAPES = [  # name, ta, tb, m, n, k
    ("xproj NT L0", 0, 1, TN, 2400, 1312),
    ("xproj NT", 0, 1, TN, 2400, 800),
    ("dX NN", 0, 0, TN, 800, 2400),
    ("dW TN", 1, 0, 2400, 800, TN),
    ("dW_ih L0 TN", 1, 0, 2400, 1312, TN),
]


def timeit(fn, iters=20):
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


def main():
    variants = sys.argv[1:] or ["plan"]
    torch.manual_seed(0)
    for name, ta, tb, m, n, k in SHAPES:
        a = torch.randn((k, m) if ta else (m, k), device=dev)
        b = torch.randn((n, k) if tb else (k, n), device=dev)
        c = torch.empty(m, n, device=dev)
        kw = dict(m=m, n=n, k=k, trans_a=bool(ta), trans_b=bool(tb), lda=a.shape[1],
                  ldb=b.shape[1], ldc=n)
        fl = 2.0 * m * n * k
        at = a.t() if ta else a
        bt = b.t() if tb else b
        tt = timeit(lambda: torch.mm(at, bt))
        ref = torch.mm(at, bt)
        line = f"{name:12s} {m:6d}x{n:5d}x{k:6d}  torch {fl / tt / 1e9:6.1f} TF |"
        for v in variants:
            os.environ.pop("DS2_GEMM_BN", None)
            os.environ.pop("DS2_GEMM_DB", None)
            if v != "plan":
                bn, db = v.split(":")
                os.environ["DS2_GEMM_BN"] = bn
                os.environ["DS2_GEMM_DB"] = db
            t32 = timeit(lambda: ops.sgemm(a, b, c, **kw))
            err = (c - ref).abs().max().item() / ref.abs().max().item()
            ours = fl / t32 / 1e9
            line += f" {v} {ours:6.1f} TF ({ours / PEAK:4.0%}, {t32 * 1e3:6.1f} us, rel {err:.0e}) |"
        print(line, flush=True)


if __name__ == "__main__":
    main()
