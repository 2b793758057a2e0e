"""Diagnostic: why conv1 on the bf16x6 kernel is opt-in (DS2_CONV_X6=2).  On the tiny golden
batch (tests/golden/tiny_ds2.npz) the train step's grad norm under DS2_CONV_X6=2 (conv1 too)
vs 1 (conv1 on the fp32 kernel), the per-parameter gradient differences, conv1 alone and the
conv1 block alone (both ~1e-6 relative), the fp32 path's sensitivity to ~1e-6 weight
perturbations, and the hardtanh inputs of the conv stack that land on the other side of 0
(one element: 4.6e-6 vs 0 -- its gradient path moves the conv gradients by ~1 %).
usage: python scripts/golden_gn_probe.py [tiny_ds2.npz]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from test_gpu_model import build_tiny, LABELS  # noqa: E402
from ds2amd.trainer import Trainer  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "tiny_ds2.npz"
g = np.load(os.path.join(REPO, "tests", "golden", name))
dev = torch.device("cuda")
res = {}
for mode in ("2", "1"):
    os.environ["DS2_CONV_X6"] = mode
    m = build_tiny(g)
    tr = Trainer(m, LABELS, lr=3e-4, momentum=0.9, max_norm=100.0, device=dev)
    data = (torch.from_numpy(g['x']), torch.from_numpy(g['targets']), None,
            torch.from_numpy(g['pct']).clone(), torch.from_numpy(g['target_sizes']))
    loss = tr.train_batch(data, return_item=True)
    gn = float(tr.optimizer.norm.item())
    grads = {k: p.grad.detach().double().cpu().clone() for k, p in m.named_parameters() if p.grad is not None}
    res[mode] = (loss, gn, grads)
    print(f"x6={mode}: loss {loss:.7f} (ref {float(g['loss']):.7f}) gn {gn:.5f} (ref {float(g['grad_norm']):.5f})")
for k in res["2"][2]:
    a, b = res["2"][2][k], res["1"][2][k]
    d = (a - b).norm().item()
    print(f"{k:40s} |g| {b.norm().item():12.4f} |dg| {d:.3e}")

# conv1 forward alone on the golden input: bf16x6 vs fp32 kernel
from ds2amd import ops  # noqa: E402
m = build_tiny(g).to(dev)
w1 = m.conv.seq_module[0].weight.detach()
b1 = m.conv.seq_module[0].bias.detach()
x = torch.from_numpy(g['x']).to(dev)
print("x", tuple(x.shape), "w1", tuple(w1.shape))
outs = {}
for mode in ("2", "1"):
    os.environ["DS2_CONV_X6"] = mode
    outs[mode] = ops.conv2d_fwd(x, w1, b1, (2, 2), (20, 5))
d = (outs["2"] - outs["1"]).abs()
print("conv1 fwd max|diff|", d.max().item(), "max|y|", outs["1"].abs().max().item(),
      "argmax", np.unravel_index(int(d.argmax()), tuple(d.shape)))

# conditioning: the fp32 kernels with conv1's weights perturbed by ~1e-7 relative
os.environ["DS2_CONV_X6"] = "1"
for eps in (1e-7, 1e-6):
    m = build_tiny(g)
    with torch.no_grad():
        w = m.conv.seq_module[0].weight
        w.mul_(1 + eps * torch.randn(w.shape, generator=torch.Generator().manual_seed(5)))
    tr = Trainer(m, LABELS, lr=3e-4, momentum=0.9, max_norm=100.0, device=dev)
    data = (torch.from_numpy(g['x']), torch.from_numpy(g['targets']), None,
            torch.from_numpy(g['pct']).clone(), torch.from_numpy(g['target_sizes']))
    loss = tr.train_batch(data, return_item=True)
    print(f"conv1 fp32, w x (1 + {eps:g} N(0,1)): loss {loss:.7f} gn {float(tr.optimizer.norm.item()):.5f}")

# conv1 block (conv -> mask -> BN -> mask -> hardtanh) fwd + bwd in isolation
m = build_tiny(g).to(dev)
conv, bn = m.conv.seq_module[0], m.conv.seq_module[1]
lens = torch.tensor([64, 50, 33], dtype=torch.int32, device=dev)
ow = (64 + 10 - 11) // 2 + 1
olens = torch.tensor([ow, (50 + 10 - 11) // 2 + 1, (33 + 10 - 11) // 2 + 1], dtype=torch.int32, device=dev)
dy = torch.randn(3, 32, 81, ow, generator=torch.Generator().manual_seed(3)).to(dev)
res2 = {}
for mode in ("2", "1"):
    os.environ["DS2_CONV_X6"] = mode
    ps = [t.detach().clone().requires_grad_(True) for t in (x, conv.weight, conv.bias, bn.weight, bn.bias)]
    rm, rv = torch.zeros(32, device=dev), torch.ones(32, device=dev)
    y = ops.ConvBlockFn.apply(ps[0], olens, ps[1], ps[2], ps[3], ps[4], rm, rv, True, 0.1, 1e-5,
                              (2, 2), (20, 5), 0.0, 20.0, 0)
    y.backward(dy)
    res2[mode] = [y.detach()] + [p.grad for p in ps[1:]]
for nm, a, b in zip(["y", "dw", "db", "dgamma", "dbeta"], res2["2"], res2["1"]):
    print(f"block {nm}: max|diff| {(a - b).abs().max().item():.3e} max|ref| {b.abs().max().item():.3e}")

# where do the two conv1 block outputs differ?  clip-boundary flips (one side exactly 0 / 20)
a, b = res2["2"][0], res2["1"][0]
flip = ((a == 0) != (b == 0)) | ((a == 20) != (b == 20))
print("block y: elements", a.numel(), "clip flips", int(flip.sum()), "zeros", int((b == 0).sum()))
d = (a - b).abs()
print("block y |diff| quantiles", [f"{q:.2e}" for q in torch.quantile(d.flatten()[:1 << 20].float(), torch.tensor([0.5, 0.9, 0.99, 0.999], device=dev)).tolist()])

# the model's whole conv stack on the golden batch: clip flips in its output
outs3 = {}
for mode in ("2", "1"):
    os.environ["DS2_CONV_X6"] = mode
    m = build_tiny(g).to(dev).train()
    lengths = torch.from_numpy(g['pct']).clone().mul_(int(x.shape[3])).int()
    olen = m.get_seq_lens(lengths).to(dev)
    with torch.no_grad():
        outs3[mode] = m.conv.forward_collapsed(x, olen)
a, b = outs3["2"], outs3["1"]
flip = ((a == 0) != (b == 0)) | ((a == 20) != (b == 20))
print("conv stack: elements", a.numel(), "clip flips", int(flip.sum()), "max|diff|", (a - b).abs().max().item())
if flip.any():
    idx = flip.nonzero()[:5]
    for i in idx.tolist():
        print("  flip at", i, float(a[tuple(i)]), float(b[tuple(i)]))
