"""conv2 of the headline model (32 x [32, 81, 501] -> 32 channels, 21 x 11 taps, stride
(2, 1)) forward, dgrad and wgrad: the bf16x6 kernels (default) vs the fp32 LDS-patch
kernels (DS2_CONV_X6=0); TFLOP/s of the algorithmic 2 * taps * in_ch * outputs.
usage: python scripts/bench_conv_x6.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
from ds2amd import ops  # noqa: E402

dev = torch.device("cuda")
n, ci, h, w, co, kh, kw, sh, sw, ph, pw = 32, 32, 81, 501, 32, 21, 11, 2, 1, 10, 5
x = torch.randn(n, ci, h, w, device=dev)
wt = torch.randn(co, ci, kh, kw, device=dev) * 0.1
ho, wo = (h + 2 * ph - kh) // sh + 1, (w + 2 * pw - kw) // sw + 1
dy = torch.randn(n, co, ho, wo, device=dev)
flop = 2.0 * kh * kw * ci * co * n * ho * wo


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


# conv1: 32 x [1, 161, 1001] -> 32 channels, 41 x 11 taps, stride (2, 2)
x1 = torch.randn(n, 1, 161, 1001, device=dev)
w1 = torch.randn(co, 1, 41, 11, device=dev) * 0.1
flop1 = 2.0 * 41 * 11 * co * n * 81 * 501

for mode in ("2", "1", "0"):   # 2: + conv1 on the bf16x6 kernel (opt-in)
    os.environ["DS2_CONV_X6"] = mode
    t1 = timeit(lambda: ops.conv2d_fwd(x1, w1, None, (2, 2), (20, 5)))
    print(f"x6={mode}: conv1 fwd {t1:.3f} ms ({flop1 / t1 / 1e9:.1f} TF)", flush=True)
    if mode == "2":
        continue
    tf = timeit(lambda: ops.conv2d_fwd(x, wt, None, (sh, sw), (ph, pw)))
    td = timeit(lambda: ops.conv2d_dgrad(dy, wt, x.shape, (sh, sw), (ph, pw)))
    tw = timeit(lambda: ops.conv2d_wgrad(dy, x, tuple(wt.shape), (sh, sw), (ph, pw), with_bias=False))
    print(f"x6={mode}: fwd {tf:.3f} ms ({flop / tf / 1e9:.1f} TF)  dgrad {td:.3f} ms "
          f"({flop / td / 1e9:.1f} TF)  wgrad {tw:.3f} ms ({flop / tw / 1e9:.1f} TF)", flush=True)
