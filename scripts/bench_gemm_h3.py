"""fp16x3 vs bf16x6 GEMM (ds2_sgemm_ws, DS2_GEMM_H3=1 vs default) on the headline step's GEMM
shapes: time (including the fp16x3 row-max pre-pass), TFLOP/s, and two errors against an fp64
product on the device -- normwise max|C - C64| / max|C64| and componentwise
max |C - C64| / (|A| |B|) (the fp32 GEMM error bound's form) -- on N(0,1) operands and on
operands whose rows and columns are scaled by 10^U(-6, 6) (the row scales' reason to exist).

usage: python scripts/bench_gemm_h3.py [--rounds 2] [--shape PREFIX]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
from ds2amd import ops  # noqa: E402

dev = torch.device("cuda")
TN = 501 * 32
SHAPES = [  # name, ta, tb, m, n, k
    ("xproj NT L0", 0, 1, TN, 4800, 1312),
    ("xproj NT", 0, 1, TN, 4800, 800),
    ("dX NN", 0, 0, TN, 800, 4800),
    ("dW_ih TN", 1, 0, 4800, 800, TN),
    ("dW_ih L0 TN", 1, 0, 4800, 1312, TN),
    ("dW_hh TN", 1, 0, 2400, 800, TN - 32),
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


def errors(c, ref, bound):
    d = (c.double() - ref).abs()
    return d.max().item() / ref.abs().max().item(), (d / bound.clamp_min(1e-300)).max().item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--shape", default=None)
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
        line = f"{name:12s} {m:6d}x{n:5d}x{k:6d} |"
        for _ in range(args.rounds):
            for tag, h3 in (("x6", "0"), ("h3", "1")):
                os.environ["DS2_GEMM_H3"] = h3
                t = timeit(lambda: ops.sgemm(a, b, c, **kw), iters=30)
                line += f" {tag} {fl / t / 1e9:6.1f} TF {t * 1e3:7.1f} us |"
        # accuracy, plain and with rows / columns spread over 12 decades
        at = a.t() if ta else a
        bt = b.t() if tb else b
        for label, sa, sb in (("N(0,1)", None, None),
                              ("rows 1e+-6", torch.pow(10.0, torch.empty(m, device=dev).uniform_(-6, 6)),
                               torch.pow(10.0, torch.empty(n, device=dev).uniform_(-6, 6)))):
            a2 = a if sa is None else (a * sa[None, :] if ta else a * sa[:, None])
            b2 = b if sb is None else (b * sb[:, None] if tb else b * sb[None, :])
            at2 = a2.t() if ta else a2
            bt2 = b2.t() if tb else b2
            ref = torch.mm(at2.double(), bt2.double())
            bound = torch.mm(at2.double().abs(), bt2.double().abs())
            kw2 = dict(kw)
            res = []
            for tag, h3 in (("x6", "0"), ("h3", "1")):
                os.environ["DS2_GEMM_H3"] = h3
                ops.sgemm(a2, b2, c, **kw2)
                torch.cuda.synchronize()
                nw, cw = errors(c, ref, bound)
                res.append(f"{tag} norm {nw:.1e} comp {cw:.1e}")
            line += f" [{label}: " + ", ".join(res) + "]"
        os.environ.pop("DS2_GEMM_H3", None)
        print(line, flush=True)


if __name__ == "__main__":
    main()
