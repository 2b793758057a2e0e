import os, sys, torch, torch.nn.functional as F
sys.path.insert(0, "deepspeech.pytorch_amd")
from ds2amd import ops
dev = torch.device("cuda")
ci, co, kh, kw, sh, sw, ph, pw = 32, 32, 21, 11, 2, 1, 10, 5
for (n, h, w) in [(4, 81, 501), (2, 81, 300)]:
    g = torch.Generator().manual_seed(5)
    x = (torch.randn(n, ci, h, w, generator=g, dtype=torch.float64) * 4 + 2).clamp(0, 20)
    wt = torch.randn(co, ci, kh, kw, generator=g, dtype=torch.float64) * 0.05
    b = torch.randn(co, generator=g, dtype=torch.float64)
    ref = F.conv2d(x, wt, b, stride=(sh, sw), padding=(ph, pw))
    dy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    dref = torch.nn.grad.conv2d_input(x.shape, wt, dy, stride=(sh, sw), padding=(ph, pw))
    f32 = F.conv2d(x.float(), wt.float(), b.float(), stride=(sh, sw), padding=(ph, pw)).double()
    for mode in ("1", "0", "fp32"):
        if mode == "fp32":
            y = f32
            d = torch.nn.grad.conv2d_input(x.shape, wt.float(), dy.float(), stride=(sh, sw), padding=(ph, pw)).double()
        else:
            os.environ["DS2_CONV_2R"] = mode
            y = ops.conv2d_fwd(x.float().to(dev), wt.float().to(dev), b.float().to(dev), (sh, sw), (ph, pw)).double().cpu()
            d = ops.conv2d_dgrad(dy.float().to(dev), wt.float().to(dev), x.shape, (sh, sw), (ph, pw)).double().cpu()
        e = y - ref; ed = d - dref
        print(f"n{n} w{w} {mode:5s} fwd max {e.abs().max().item()/ref.abs().max().item():.2e} rms {e.pow(2).mean().sqrt().item()/ref.pow(2).mean().sqrt().item():.2e} drift {(e.mean()/e.abs().mean()).item():+.3f} | dgrad max {ed.abs().max().item()/dref.abs().max().item():.2e} rms {ed.pow(2).mean().sqrt().item()/dref.pow(2).mean().sqrt().item():.2e} drift {(ed.mean()/ed.abs().mean()).item():+.3f}", flush=True)
