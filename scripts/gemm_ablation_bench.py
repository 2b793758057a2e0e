"""Timing of the bf16x6 GEMM on the step's shapes with whichever libds2hip.so DS2_LIB_PATH names
(scripts/gemm_ablation.sh builds the ablation variants; their results are not checked).

usage: DS2_LIB_PATH=... python scripts/gemm_ablation_bench.py TAG
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
from ds2amd import ops  # noqa: E402

dev = torch.device("cuda")
TN = 501 * 32
SHAPES = [("xproj NT L0", 0, 1, TN, 4800, 1312), ("dX NN", 0, 0, TN, 800, 4800),
          ("dW_ih TN", 1, 0, 4800, 800, TN), ("dW_hh TN", 1, 0, 2400, 800, TN - 32)]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "base"
    torch.manual_seed(0)
    line = f"{tag:6s}"
    for name, ta, tb, m, n, k in SHAPES:
        a = torch.randn((k, m) if ta else (m, k), device=dev)
        b = torch.randn((n, k) if tb else (k, n), device=dev)
        c = torch.empty(m, n, device=dev)
        kw = dict(m=m, n=n, k=k, trans_a=bool(ta), trans_b=bool(tb), lda=a.shape[1],
                  ldb=b.shape[1], ldc=n)
        for _ in range(3):
            ops.sgemm(a, b, c, **kw)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(30):
            ops.sgemm(a, b, c, **kw)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 30
        line += f" | {name} {t * 1e3:7.1f} us {2.0 * m * n * k / t / 1e9:6.1f} TF"
    print(line, flush=True)


if __name__ == "__main__":
    main()
