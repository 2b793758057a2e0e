"""Microbenchmark: the model's two convolutions (fwd, dgrad, wgrad) through the ds2 ops,
TFLOP/s per pass (2 * N * Co * Ho * Wo * Ci * kh * kw each)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
from ds2amd import ops  # noqa: E402

dev = torch.device("cuda")
CONVS = [("conv1", 32, 1, 161, 1001, 32, 41, 11, 2, 2, 20, 5),
         ("conv2", 32, 32, 81, 501, 32, 21, 11, 2, 1, 10, 5)]


def timeit(fn, iters=5):
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


for name, n, ci, h, w, co, kh, kw, sh, sw, ph, pw in CONVS:
    ho, wo = ops.conv_out_shape(h, w, kh, kw, sh, sw, ph, pw)
    x = torch.randn(n, ci, h, w, device=dev)
    wt = torch.randn(co, ci, kh, kw, device=dev) * 0.05
    b = torch.randn(co, device=dev)
    dy = torch.randn(n, co, ho, wo, device=dev)
    fl = 2.0 * n * co * ho * wo * ci * kh * kw
    tf = timeit(lambda: ops.conv2d_fwd(x, wt, b, (sh, sw), (ph, pw)))
    out = [f"fwd {tf * 1e3:7.1f} us {fl / tf / 1e9:6.1f} TF"]
    if ci > 1:
        td = timeit(lambda: ops.conv2d_dgrad(dy, wt, x.shape, (sh, sw), (ph, pw)))
        out.append(f"dgrad {td * 1e3:7.1f} us {fl / td / 1e9:6.1f} TF")
    # no bias gradient: the training step takes the conv bias gradient from the BN backward
    tw = timeit(lambda: ops.conv2d_wgrad(dy, x, wt.shape, (sh, sw), (ph, pw), False))
    out.append(f"wgrad {tw * 1e3:7.1f} us {fl / tw / 1e9:6.1f} TF")
    print(f"{name}: " + " | ".join(out), flush=True)
