"""Systematic (non-cancelling) error of the conv2 kernels, the quantity the BatchNorm
parameter gradients of the conv block amplify: dbeta = sum over positions of dy and dgamma =
sum of dy x_hat are sums of 1.3 M terms that nearly cancel (dy comes out of the next
BatchNorm's backward, zero-mean per channel), so per-element errors that share a sign survive
the sum while random ones cancel.

For conv2's shape (32 -> 32 channels, 21 x 11 taps, stride (2, 1)) at a reduced batch this
prints, per kernel mode (h3: fp16x3, its small products in their own MFMA chain; x6: bf16x6;
fp32 -- DS2_CONV_H3 / DS2_CONV_X6) and direction (forward
y, dgrad dx), the max elementwise error relative to max |ref| and the per-channel SUM error
relative to the channel's sum of |ref|, against an fp64 torch reference on the same fp32
inputs.  dy is made zero-mean per channel, as a BatchNorm backward leaves it.

usage: python scripts/conv_bias_probe.py [--n 4] [--w 501]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from ds2amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4)
    ap.add_argument("--w", type=int, default=501)
    args = ap.parse_args()
    dev = torch.device("cuda")
    n, ci, h, w, co, kh, kw, sh, sw, ph, pw = args.n, 32, 81, args.w, 32, 21, 11, 2, 1, 10, 5
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(n, ci, h, w, generator=g) * 20).float()            # hardtanh(0, 20) outputs
    wt = (torch.randn(co, ci, kh, kw, generator=g) * (ci * kh * kw) ** -0.5).float()
    y64 = F.conv2d(x.double(), wt.double(), None, stride=(sh, sw), padding=(ph, pw))
    dy = torch.randn(y64.shape, generator=g, dtype=torch.float64)
    dy = (dy - dy.mean((0, 2, 3), keepdim=True)).float()
    dx64 = torch.nn.grad.conv2d_input(x.shape, wt.double(), dy.double(), stride=(sh, sw),
                                      padding=(ph, pw))
    for mode in ("h3", "x6", "fp32"):
        os.environ["DS2_CONV_X6"] = "0" if mode == "fp32" else "1"
        os.environ["DS2_CONV_H3"] = "1" if mode == "h3" else "0"
        yd = ops.conv2d_fwd(x.to(dev), wt.to(dev), None, (sh, sw), (ph, pw)).double().cpu()
        dx = ops.conv2d_dgrad(dy.to(dev), wt.to(dev), x.shape, (sh, sw), (ph, pw)).double().cpu()
        for name, a, r in (("fwd y", yd, y64), ("dgrad dx", dx, dx64)):
            el = (a - r).abs().max().item() / r.abs().max().item()
            s_err = ((a - r).sum((0, 2, 3)).abs() / r.abs().sum((0, 2, 3))).max().item()
            s_rel = ((a - r).sum((0, 2, 3)).abs() / r.sum((0, 2, 3)).abs().clamp_min(1e-300)).max().item()
            # a sign test of the per-element error: mean(err) / mean(|err|)
            e = a - r
            bias = (e.mean() / e.abs().mean().clamp_min(1e-300)).item()
            print(f"{mode:8s} {name:9s} elem {el:.2e}  chan-sum err/sum|ref| {s_err:.2e}  "
                  f"chan-sum rel {s_rel:.2e}  mean(err)/mean|err| {bias:+.3f}", flush=True)


if __name__ == "__main__":
    main()
