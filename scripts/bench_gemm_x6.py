"""Microbenchmark + accuracy: ds2_sgemm_ws on the bf16x6 kernel (default) vs the fp32-MFMA
kernel (DS2_GEMM_X6=0) on the headline step's GEMM shapes (5 x BiGRU-800, batch 32,
T' = 501: TN = 16032 rows).  Error = max |C - C_fp64| / max |C_fp64| for both kernels, with
the fp64 product computed by torch on the device.  Prints TFLOP/s and the fraction of the
fp32-equivalent peak each kernel runs against (fp32 MFMA 157.3 TF; bf16x6 2516.6 / 6 TF).

usage: python scripts/bench_gemm_x6.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
from ds2amd import ops  # noqa: E402

dev = torch.device("cuda")
TN = 501 * 32
PEAK32, PEAKX6 = 157.3, 2516.6 / 6
SHAPES = [  # name, ta, tb, m, n, k
    ("xproj NT L0", 0, 1, TN, 4800, 1312),      # both directions stacked (as in the step)
    ("xproj NT", 0, 1, TN, 4800, 800),
    ("dX NN", 0, 0, TN, 800, 4800),
    ("dW_ih TN", 1, 0, 4800, 800, TN),
    ("dW_ih L0 TN", 1, 0, 4800, 1312, TN),
    ("dW_hh TN", 1, 0, 2400, 800, TN - 32),     # one direction, T - 1 steps
    ("FC NT", 0, 1, TN, 32, 800),
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
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default=None, help="one shape (name prefix), e.g. for rocprofv3")
    ap.add_argument("--mode", default=None, choices=["x6", "fp32"])
    args = ap.parse_args()
    torch.manual_seed(0)
    for name, ta, tb, m, n, k in SHAPES:
        if args.shape is not None and not name.startswith(args.shape):
            continue
        a = torch.randn((k, m) if ta else (m, k), device=dev)
        b = torch.randn((n, k) if tb else (k, n), device=dev)
        c = torch.empty(m, n, device=dev)
        kw = dict(m=m, n=n, k=k, trans_a=bool(ta), trans_b=bool(tb), lda=a.shape[1],
                  ldb=b.shape[1], ldc=n)
        fl = 2.0 * m * n * k
        at = a.t() if ta else a
        bt = b.t() if tb else b
        ref = torch.mm(at.double(), bt.double())
        scale = ref.abs().max().item()
        line = f"{name:12s} {m:6d}x{n:5d}x{k:6d} |"
        # alternating twice (the clock the chip holds differs by body)
        for tag, env, peak in (("x6", "1", PEAKX6), ("x6", "1", PEAKX6), ("fp32", "0", PEAK32)):
            if args.mode is not None and tag != args.mode:
                continue
            os.environ["DS2_GEMM_X6"] = env
            t = timeit(lambda: ops.sgemm(a, b, c, **kw), iters=30)
            err = (c.double() - ref).abs().max().item() / scale
            tf = fl / t / 1e9
            line += f" {tag} {tf:6.1f} TF ({tf / peak:4.0%}) {t * 1e3:7.1f} us err {err:.1e} |"
        os.environ.pop("DS2_GEMM_X6", None)
        print(line, flush=True)


if __name__ == "__main__":
    main()
