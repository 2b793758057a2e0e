"""How much of the conv block's BatchNorm-gradient distance comes from representing conv2's
weights in two fp16 terms (fp16x3 / "h3": hi + lo carry ~23 of fp32's 24 significant bits,
so every weight is off by up to ~1 fp32 ulp, the same weights at every position).

CPU only.  The conv block (model.py:208-215, all lengths full so MaskConv is the identity)
runs in fp64 with conv2's weight W replaced by its h3 image hi + lo (row-scaled by the
output channel's max, as the kernels do) in the forward, the dgrad, or both, and in fp32
(the oracle's arithmetic); each run reuses the exact fp64 run's Hardtanh masks, as the bs32
test does, and prints each conv parameter's gradient distance from the exact fp64 run
(max-abs / max-abs).

usage: python scripts/conv_weight_split_probe.py [--n 4] [--seed 13]
"""
import argparse

import torch
import torch.nn.functional as F

P = ['w1', 'b1', 'g1', 'be1', 'w2', 'b2', 'g2', 'be2']


def h3_image(w):
    """hi + lo of the per-output-channel scaled fp16 split (csrc/rnn_common.h split2h)."""
    w = w.float()
    amax = w.abs().flatten(1).amax(1).clamp_min(1e-30)
    e = 14 - torch.floor(torch.log2(amax))
    sc = torch.pow(2.0, e).view(-1, *([1] * (w.dim() - 1)))
    ws = w * sc
    hi = ws.half()
    lo = (ws - hi.float()).half()
    return ((hi.double() + lo.double()) / sc.double())


class Conv2Split(torch.autograd.Function):
    """conv2 with one weight in the forward and another in the dgrad (wgrad exact)."""

    @staticmethod
    def forward(ctx, x, w, b, w_fwd, w_bwd):
        ctx.save_for_backward(x, w, w_bwd)
        return F.conv2d(x, w_fwd, b, stride=(2, 1), padding=(10, 5))

    @staticmethod
    def backward(ctx, gy):
        x, w, w_bwd = ctx.saved_tensors
        dx = torch.nn.grad.conv2d_input(x.shape, w_bwd, gy, stride=(2, 1), padding=(10, 5))
        dw = torch.nn.grad.conv2d_weight(x, w.shape, gy, stride=(2, 1), padding=(10, 5))
        return dx, dw, gy.sum((0, 2, 3)), None, None


def bn(x, g, b):
    mu = x.mean((0, 2, 3), keepdim=True)
    var = x.var((0, 2, 3), unbiased=False, keepdim=True)
    return (x - mu) / torch.sqrt(var + 1e-5) * g.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)


def htanh(x, mask):
    if mask is None:
        return F.hardtanh(x, 0, 20)
    return F.hardtanh(x, 0, 20).detach() + mask.to(x.dtype) * (x - x.detach())


def block(p, x, g_out, dtype, masks=None, w2_fwd=None, w2_bwd=None):
    q = {k: v.to(dtype).clone().requires_grad_(True) for k, v in p.items()}
    y = F.conv2d(x.to(dtype), q['w1'], q['b1'], stride=(2, 2), padding=(20, 5))
    z1 = bn(y, q['g1'], q['be1'])
    a1 = htanh(z1, None if masks is None else masks[0])
    wf = q['w2'] if w2_fwd is None else w2_fwd.to(dtype)
    wb = q['w2'].detach() if w2_bwd is None else w2_bwd.to(dtype)
    y2 = Conv2Split.apply(a1, q['w2'], q['b2'], wf, wb)
    z2 = bn(y2, q['g2'], q['be2'])
    a2 = htanh(z2, None if masks is None else masks[1])
    n, c, d, t = a2.shape
    out = a2.view(n, c * d, t).permute(2, 0, 1)
    out.backward(g_out.to(dtype))
    m = ((z1 > 0) & (z1 < 20)).detach(), ((z2 > 0) & (z2 < 20)).detach()
    return {k: v.grad.double() for k, v in q.items()}, m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4)
    ap.add_argument("--seed", type=int, default=13)
    args = ap.parse_args()
    g = torch.Generator().manual_seed(args.seed)
    n = args.n
    x = torch.randn(n, 1, 161, 1001, generator=g)
    p = {'w1': torch.randn(32, 1, 41, 11, generator=g) * (451 ** -0.5),
         'b1': torch.randn(32, generator=g) * 0.05,
         'g1': torch.ones(32), 'be1': torch.zeros(32),
         'w2': torch.randn(32, 32, 21, 11, generator=g) * (7392 ** -0.5),
         'b2': torch.randn(32, generator=g) * 0.05,
         'g2': torch.ones(32), 'be2': torch.zeros(32)}
    g_out = torch.randn(501, n, 32 * 41, generator=g) * 1e-3
    ref, masks = block(p, x, g_out, torch.float64)
    w2h = h3_image(p['w2'])
    print(f"h3 image of W2: max rel error {((w2h - p['w2'].double()).abs() / p['w2'].double().abs().clamp_min(1e-30)).max().item():.2e}",
          flush=True)
    runs = {
        "fp32 (oracle arithmetic)": dict(dtype=torch.float32),
        "fp64, W2 h3 fwd+dgrad": dict(dtype=torch.float64, w2_fwd=w2h, w2_bwd=w2h),
        "fp64, W2 h3 fwd only": dict(dtype=torch.float64, w2_fwd=w2h),
        "fp64, W2 h3 dgrad only": dict(dtype=torch.float64, w2_bwd=w2h),
    }
    for name, kw in runs.items():
        gr, _ = block(p, x, g_out, kw.pop('dtype'), masks, **kw)
        d = {k: ((gr[k] - ref[k]).abs().max() / ref[k].abs().max()).item() for k in P}
        print(f"{name:26s} " + "  ".join(f"{k} {v:.2e}" for k, v in d.items()), flush=True)


if __name__ == "__main__":
    main()
