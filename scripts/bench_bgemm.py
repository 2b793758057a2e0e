"""Microbenchmark: ds2_bgemm_nt (bf16 operands already in HBM, csrc/bgemm.hip) on BASELINE
cfg4's RNN GEMM shapes (7 x BiLSTM-1024, batch 64, T' = 501: TN = 32064 rows), each operand
in the k-contiguous layout the kernel reads, beside torch.mm on the same bf16 operands
(hipBLASLt, in the layout torch gets them).  Dense bf16 peak 2516.6 TF.

usage: python scripts/bench_bgemm.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
from ds2amd import ops  # noqa: E402

dev = torch.device("cuda")
TN = 501 * 64
PEAK = 2516.6
SHAPES = [  # name, m, n, k (C[m, n] = A[m, k] B[n, k]^T)
    ("xproj L0 (both dirs)", TN, 8192, 1312),
    ("xproj (both dirs)", TN, 8192, 1024),
    ("dX (both dirs)", TN, 1024, 8192),
    ("dW_ih (both dirs)", 8192, 1024, TN),
    ("dW_hh (one dir)", 4096, 1024, TN),
    ("sq 8192", 8192, 8192, 8192),
]


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


def main():
    torch.manual_seed(0)
    for name, m, n, k in SHAPES:
        a = (torch.rand(m, k, device=dev) * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(n, k, device=dev) * 2 - 1).to(torch.bfloat16)
        c = torch.empty(m, n, device=dev)
        fl = 2.0 * m * n * k
        t = timeit(lambda: ops.bgemm_nt(a, b, c))
        ref = torch.mm(a.float()[:256], b.float().t())
        err = (c[:256] - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)
        tt = timeit(lambda: torch.mm(a, b.t()))
        tf, tft = fl / t / 1e9, fl / tt / 1e9
        print(f"{name:22s} {m:6d}x{n:5d}x{k:6d}  ds2_bgemm_nt {tf:7.1f} TF ({tf / PEAK:4.0%}) "
              f"{t * 1e3:8.1f} us err {err:.1e} | torch.mm bf16 {tft:7.1f} TF ({tft / PEAK:4.0%})",
              flush=True)


if __name__ == "__main__":
    main()
