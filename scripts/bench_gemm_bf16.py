"""Microbenchmark: ds2_sgemm_bf16_ws (fp32 operands rounded to bf16 while staged, bf16 MFMA,
fp32 accumulate) on BASELINE cfg4's RNN GEMM shapes (7 x BiLSTM-1024, batch 64, T' = 501)
vs our fp32 GEMM and vs torch.mm on operands already in bf16 (hipBLASLt; conversion not
timed)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
from ds2amd import ops  # noqa: E402

dev = torch.device("cuda")
TN = 501 * 64
SHAPES = [  # name, ta, tb, m, n, k
    ("xproj NT L0", 0, 1, TN, 4096, 1312),
    ("xproj NT", 0, 1, TN, 4096, 1024),
    ("dX NN", 0, 0, TN, 1024, 4096),
    ("dW_ih TN", 1, 0, 4096, 1024, TN),
    ("sq NN", 0, 0, 4096, 4096, 4096),
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


for name, ta, tb, m, n, k in SHAPES:
    a = torch.randn((k, m) if ta else (m, k), device=dev)
    b = torch.randn((n, k) if tb else (k, n), device=dev)
    c = torch.empty(m, n, device=dev)
    kw = dict(m=m, n=n, k=k, trans_a=bool(ta), trans_b=bool(tb), lda=a.shape[1],
              ldb=b.shape[1], ldc=n)
    fl = 2.0 * m * n * k
    t16 = timeit(lambda: ops.sgemm(a, b, c, bf16=True, **kw))
    t32 = timeit(lambda: ops.sgemm(a, b, c, **kw))
    ab, bb = a.to(torch.bfloat16), b.to(torch.bfloat16)
    at = ab.t() if ta else ab
    bt = bb.t() if tb else bb
    tt = timeit(lambda: torch.mm(at, bt))
    print(f"{name:12s} {m:6d}x{n:5d}x{k:6d}  ours bf16 {fl / t16 / 1e9:7.1f} TF  "
          f"ours fp32 {fl / t32 / 1e9:6.1f} TF  torch bf16 (hipBLASLt) {fl / tt / 1e9:7.1f} TF",
          flush=True)
