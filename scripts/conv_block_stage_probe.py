"""Which stage of the conv block puts its error into the first BatchNorm's gradients?

The bs32 train-step test compares the conv block's parameter gradients with an fp64 run of
the same block (same upstream gradient, same Hardtanh masks).  BN1's gamma / beta gradients
are sums over 1.3 M positions per channel of a gradient that nearly cancels, so they
amplify any error that is correlated over positions.  This probe runs the block's two
layers (conv -> BN -> Hardtanh, ops.ConvBlockFn) separately on the GPU, each fed the exact
(fp64, rounded to fp32) input / upstream gradient, and prints BN1's gradient distance from
the exact run caused by
  layer 2 (conv2 forward, BN2 statistics + backward, conv2 dgrad), pushed through an fp64
          layer-1 backward, and
  layer 1 (conv1 forward, BN1 statistics + backward),
each next to the same split of the fp32 torch arithmetic the oracle uses.

usage: python scripts/conv_block_stage_probe.py [--n 8] [--seed 13]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from ds2amd import ops  # noqa: E402

S1, P1, S2, P2 = (2, 2), (20, 5), (2, 1), (10, 5)


def bn(x, g, b):
    mu = x.mean((0, 2, 3), keepdim=True)
    var = x.var((0, 2, 3), unbiased=False, keepdim=True)
    return (x - mu) / torch.sqrt(var + 1e-5) * g.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)


def layer_ref(x, w, b, g, be, stride, pad, mask, dtype, gy):
    """fp64 / fp32 conv -> BN -> Hardtanh with the given derivative mask; returns
    (output, dx, {w, g, be} grads)."""
    q = [t.to(dtype).detach().clone().requires_grad_(True) for t in (x, w, b, g, be)]
    z = bn(F.conv2d(q[0], q[1], q[2], stride=stride, padding=pad), q[3], q[4])
    y = F.hardtanh(z, 0, 20).detach() + mask.to(dtype) * (z - z.detach())
    y.backward(gy.to(dtype))
    return y.detach(), q[0].grad.double(), {k: v.grad.double() for k, v in
                                            zip(("w", "b", "g", "be"), q[1:])}


def layer_ours(x, w, b, g, be, stride, pad, gy, dev):
    n = x.shape[0]
    t_out = (x.shape[3] + 2 * pad[1] - w.shape[3]) // stride[1] + 1
    lens = torch.full((n,), t_out, dtype=torch.int32, device=dev)
    q = [t.float().to(dev).detach().clone().requires_grad_(True) for t in (x, w, b, g, be)]
    rm = torch.zeros(w.shape[0], device=dev)
    rv = torch.ones(w.shape[0], device=dev)
    y = ops.ConvBlockFn.apply(q[0], lens, q[1], q[2], q[3], q[4], rm, rv, True, 0.1, 1e-5,
                              stride, pad, 0.0, 20.0, 0)
    y.backward(gy.float().to(dev))
    return y.detach().cpu(), q[0].grad.double().cpu(), {
        k: v.grad.double().cpu() for k, v in zip(("w", "b", "g", "be"), q[1:])}


def dist(a, r):
    return ((a - r).abs().max() / r.abs().max()).item()


def _report_err(name, a, r, m):
    """conv2 dgrad error structure: elementwise, bias, the masked per-channel sums BN1 takes,
    correlation with the result, and the error's mean over the edge / middle columns."""
    e = a - r
    el = (e.abs().max() / r.abs().max()).item()
    bias = (e.mean() / e.abs().mean()).item()
    ms = ((m * e).sum((0, 2, 3)).abs() / (m * r).sum((0, 2, 3)).abs()).max().item()
    ms_abs = ((m * e).sum((0, 2, 3)).abs() / (m * r).abs().sum((0, 2, 3))).max().item()
    corr = ((e * r).sum() / (e.square().sum() * r.square().sum()).sqrt()).item()
    w = e.shape[3]
    col = e.mean((0, 1, 2)) / e.abs().mean()
    row = e.mean((0, 1, 3)) / e.abs().mean()
    print(f"  dgrad {name:11s}: elem {el:.2e}  mean(e)/mean|e| {bias:+.3f}  corr(e, dx) {corr:+.3f}"
          f"  masked chan-sum err / |sum| {ms:.2e}  / sum|.| {ms_abs:.2e}"
          f"  col-mean e (first 6 / mid / last 6) {[round(v, 3) for v in col[:6].tolist()]}"
          f" {col[6:w - 6].abs().max().item():.3f} {[round(v, 3) for v in col[-6:].tolist()]}"
          f"  row-mean max {row.abs().max().item():.3f}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--seed", type=int, default=13)
    args = ap.parse_args()
    torch.set_num_threads(max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or 16))))
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(args.seed)
    n = args.n
    x = torch.randn(n, 1, 161, 1001, generator=g)
    w1 = torch.randn(32, 1, 41, 11, generator=g) * (451 ** -0.5)
    b1 = torch.randn(32, generator=g) * 0.05
    w2 = torch.randn(32, 32, 21, 11, generator=g) * (7392 ** -0.5)
    b2 = torch.randn(32, generator=g) * 0.05
    ga, be = torch.ones(32), torch.zeros(32)
    # exact forward: masks and the layer-1 output
    with torch.no_grad():
        z1 = bn(F.conv2d(x.double(), w1.double(), b1.double(), stride=S1, padding=P1), ga.double(),
                be.double())
        m1 = (z1 > 0) & (z1 < 20)
        a1 = F.hardtanh(z1, 0, 20)
        z2 = bn(F.conv2d(a1, w2.double(), b2.double(), stride=S2, padding=P2), ga.double(),
                be.double())
        m2 = (z2 > 0) & (z2 < 20)
    gy2 = torch.randn(z2.shape, generator=g, dtype=torch.float64) * 1e-3
    a1f = a1.float()
    # layer 2 alone, exact input a1 (fp32-rounded); the references use our Hardtanh mask
    y2, da1_o, gr2_o = layer_ours(a1f, w2, b2, ga, be, S2, P2, gy2, dev)
    m2o = (y2 > 0) & (y2 < 20)
    print(f"n {n}: layer-2 mask flips vs exact forward {(m2o != m2).sum().item()}", flush=True)
    _, da1_64, g2_64 = layer_ref(a1, w2, b2, ga, be, S2, P2, m2o, torch.float64, gy2)
    _, _, g1_64 = layer_ref(x, w1, b1, ga, be, S1, P1, m1, torch.float64, da1_64)
    _, da1_32, gr2_32 = layer_ref(a1f, w2, b2, ga, be, S2, P2, m2o, torch.float32, gy2)
    for name, da1, gr2 in (("ours", da1_o, gr2_o), ("fp32 torch", da1_32, gr2_32)):
        # BN1 gradient error this layer-2 error causes: exact layer-1 backward of da1
        _, _, g1 = layer_ref(x, w1, b1, ga, be, S1, P1, m1, torch.float64, da1)
        print(f"layer 2 {name:10s}: d a1 {dist(da1, da1_64):.2e}  w2 {dist(gr2['w'], g2_64['w']):.2e}"
              f"  g2 {dist(gr2['g'], g2_64['g']):.2e}  be2 {dist(gr2['be'], g2_64['be']):.2e}"
              f"  -> BN1 g1 {dist(g1['g'], g1_64['g']):.2e}  be1 {dist(g1['be'], g1_64['be']):.2e}"
              f"  w1 {dist(g1['w'], g1_64['w']):.2e}", flush=True)
    # layer 2 stage by stage: each of our kernels on exact (fp32-rounded) inputs, the rest fp64
    def bn1_err(da1):
        _, _, g1 = layer_ref(x, w1, b1, ga, be, S1, P1, m1, torch.float64, da1)
        return f"BN1 g1 {dist(g1['g'], g1_64['g']):.2e}  be1 {dist(g1['be'], g1_64['be']):.2e}"

    def bn2_bwd_ref(zpre, dtype):
        zq = zpre.to(dtype).detach().clone().requires_grad_(True)
        zz = bn(zq, ga.to(dtype), be.to(dtype))
        yy = F.hardtanh(zz, 0, 20).detach() + m2o.to(dtype) * (zz - zz.detach())
        yy.backward(gy2.to(dtype))
        return zq.grad.double()

    z2pre = F.conv2d(a1, w2.double(), b2.double(), stride=S2, padding=P2)
    dz2_64 = bn2_bwd_ref(z2pre, torch.float64)
    nb, cb, db, tb = z2pre.shape
    lens = torch.full((nb,), tb, dtype=torch.int32, device=dev)
    # (A) conv2 dgrad alone
    dx = ops.conv2d_dgrad(dz2_64.float().to(dev), w2.float().to(dev), a1.shape, S2, P2)
    print(f"  conv2 dgrad ours      : {bn1_err(dx.double().cpu())}", flush=True)
    dx = torch.nn.grad.conv2d_input(a1.shape, w2.float(), dz2_64.float(), stride=S2, padding=P2)
    print(f"  conv2 dgrad fp32 torch: {bn1_err(dx.double())}", flush=True)

    # the structure of conv2 dgrad's error, per conv mode
    dx64 = torch.nn.grad.conv2d_input(a1.shape, w2.double(), dz2_64.float().double(), stride=S2,
                                      padding=P2)
    m1d = m1.double()
    for mode in ("h3", "x6", "fp32"):
        os.environ["DS2_CONV_X6"] = "0" if mode == "fp32" else "1"
        os.environ["DS2_CONV_H3"] = "1" if mode == "h3" else "0"
        dx = ops.conv2d_dgrad(dz2_64.float().to(dev), w2.float().to(dev), a1.shape, S2,
                              P2).double().cpu()
        _report_err(f"ours {mode}", dx, dx64, m1d)
    os.environ["DS2_CONV_X6"] = "1"
    os.environ["DS2_CONV_H3"] = "1"
    dx = torch.nn.grad.conv2d_input(a1.shape, w2.float(), dz2_64.float(), stride=S2,
                                    padding=P2).double()
    _report_err("fp32 torch", dx, dx64, m1d)

    def dgrad64(dz):
        return torch.nn.grad.conv2d_input(a1.shape, w2.double(), dz, stride=S2, padding=P2)
    # (B) BN2 statistics + backward alone (on the exact conv2 output)
    zf = z2pre.float().to(dev).contiguous()
    mean, invstd = ops.bn_stats(zf, nb, cb, db * tb, 1e-5, 0.1, torch.zeros(cb, device=dev),
                                torch.ones(cb, device=dev), True)
    dz, _, _, _ = ops.bn_backward(gy2.float().to(dev).contiguous(), 0, zf, nb, cb, db, tb, mean,
                                  invstd, ga.float().to(dev), be.float().to(dev), masked=True,
                                  lens=lens, lo=0.0, hi=20.0)
    print(f"  BN2 stats+bwd ours    : dz2 {dist(dz.double().cpu(), dz2_64):.2e}  "
          f"{bn1_err(dgrad64(dz.double().cpu()))}", flush=True)
    dz = bn2_bwd_ref(z2pre.float(), torch.float32)
    print(f"  BN2 stats+bwd fp32    : dz2 {dist(dz, dz2_64):.2e}  {bn1_err(dgrad64(dz))}",
          flush=True)
    # (C) conv2 forward alone (its output through the exact BN2 backward)
    zo = ops.conv2d_fwd(a1f.to(dev), w2.float().to(dev), b2.float().to(dev), S2, P2)
    dz = bn2_bwd_ref(zo.double().cpu(), torch.float64)
    print(f"  conv2 fwd ours        : z2 {dist(zo.double().cpu(), z2pre):.2e}  "
          f"{bn1_err(dgrad64(dz))}", flush=True)
    zo = F.conv2d(a1f, w2.float(), b2.float(), stride=S2, padding=P2)
    dz = bn2_bwd_ref(zo.double(), torch.float64)
    print(f"  conv2 fwd fp32 torch  : z2 {dist(zo.double(), z2pre):.2e}  "
          f"{bn1_err(dgrad64(dz))}", flush=True)
    # layer 1 alone, exact upstream gradient (fp32-rounded), references on our mask
    da1f = da1_64.float()
    y1, _, gr1_o = layer_ours(x, w1, b1, ga, be, S1, P1, da1f, dev)
    m1o = (y1 > 0) & (y1 < 20)
    print(f"layer-1 mask flips vs exact forward {(m1o != m1).sum().item()}", flush=True)
    _, _, g1r = layer_ref(x, w1, b1, ga, be, S1, P1, m1o, torch.float64, da1_64)
    _, _, gr1_32 = layer_ref(x, w1, b1, ga, be, S1, P1, m1o, torch.float32, da1f)
    for name, gr1 in (("ours", gr1_o), ("fp32 torch", gr1_32)):
        print(f"layer 1 {name:10s}: g1 {dist(gr1['g'], g1r['g']):.2e}  be1 "
              f"{dist(gr1['be'], g1r['be']):.2e}  w1 {dist(gr1['w'], g1r['w']):.2e}", flush=True)


if __name__ == "__main__":
    main()
