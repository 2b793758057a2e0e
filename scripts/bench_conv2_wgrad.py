"""A/B: conv2's fp16x3 sliding-window weight gradient on 32-column row stages (default) vs
64-column ones (DS2_CONV_W64=1), the headline shape (32 x [32, 81, 501] -> 32 channels, 21 x 11
taps, stride (2, 1)), alternating in one process; max difference between the two.
usage: python scripts/bench_conv2_wgrad.py [rounds]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
from ds2amd import ops  # noqa: E402

dev = torch.device("cuda")
n, ci, h, w, co, kh, kw, sh, sw, ph, pw = 32, 32, 81, 501, 32, 21, 11, 2, 1, 10, 5
x = torch.rand(n, ci, h, w, device=dev) * 3
ho, wo = (h + 2 * ph - kh) // sh + 1, (w + 2 * pw - kw) // sw + 1
dy = torch.randn(n, co, ho, wo, device=dev)
flop = 2.0 * kh * kw * ci * co * n * ho * wo


def run():
    return ops.conv2d_wgrad(dy, x, (co, ci, kh, kw), (sh, sw), (ph, pw), with_bias=False)[0]


def timeit(iters=20):
    run()
    torch.cuda.synchronize()
    a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        run()
    c.record()
    torch.cuda.synchronize()
    return a.elapsed_time(c) / iters


rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
outs = {}
for r in range(rounds):
    for mode in ("0", "1"):
        os.environ["DS2_CONV_W64"] = mode
        ms = timeit()
        outs[mode] = run()
        print(f"wgrad round {r} {'64-col' if mode == '1' else '32-col'}: {ms * 1e3:8.1f} us "
              f"({flop / ms / 1e9:6.1f} TF, {flop / ms / 1e9 / 838.9:.3f} of 838.9)", flush=True)
d = (outs["1"] - outs["0"]).abs().max().item() / outs["0"].abs().max().item()
print(f"wgrad: max |64 - 32| / max |32| = {d:.2e}")
