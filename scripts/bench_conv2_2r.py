"""A/B: conv2's fp16x3 forward and dgrad with two output rows per workgroup
(conv_h3_fwd2r_kernel / conv_h3_dgrad2r_kernel, default) vs one (conv_x6_kernel /
conv_x6q_dgrad_kernel, DS2_CONV_2R=0), the headline shape (32 x [32, 81, 501] -> 32
channels, 21 x 11 taps, stride (2, 1)), alternating in one process.
usage: python scripts/bench_conv2_2r.py [rounds]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
from ds2amd import ops  # noqa: E402

dev = torch.device("cuda")
n, ci, h, w, co, kh, kw, sh, sw, ph, pw = 32, 32, 81, 501, 32, 21, 11, 2, 1, 10, 5
x = torch.rand(n, ci, h, w, device=dev) * 3
wt = torch.randn(co, ci, kh, kw, device=dev) * 0.05
b = torch.randn(co, device=dev)
ho, wo = (h + 2 * ph - kh) // sh + 1, (w + 2 * pw - kw) // sw + 1
flop = 2.0 * kh * kw * ci * co * n * ho * wo


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    c.record()
    torch.cuda.synchronize()
    return a.elapsed_time(c) / iters


rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dy = torch.randn(n, co, ho, wo, device=dev)
ops_ = {"fwd": lambda: ops.conv2d_fwd(x, wt, b, (sh, sw), (ph, pw)),
        "dgrad": lambda: ops.conv2d_dgrad(dy, wt, (n, ci, h, w), (sh, sw), (ph, pw))}
for name, fn in ops_.items():
    ys = {}
    for r in range(rounds):
        for mode in ("1", "0"):
            os.environ["DS2_CONV_2R"] = mode
            ms = timeit(fn)
            ys[mode] = fn()
            print(f"{name} round {r} {'two-row' if mode == '1' else 'one-row'}: {ms * 1e3:8.1f} us "
                  f"({flop / ms / 1e9:6.1f} TF, {flop / ms / 1e9 / 838.9:.3f} of 838.9)", flush=True)
    d = (ys["1"] - ys["0"]).abs().max().item() / ys["0"].abs().max().item()
    print(f"{name}: max |two - one| / max |one| = {d:.2e}")
