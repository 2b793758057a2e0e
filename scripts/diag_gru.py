"""Diagnostic: phase breakdown of the persistent GRU forward (DS2_GRU_STAMPS=1)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
os.environ["DS2_GRU_STAMPS"] = "1"
import torch  # noqa: E402
from ds2amd import _lib, ops  # noqa: E402

T, N, H, D = 501, 32, 800, 2
dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(0)
xproj = (torch.randn(T, N, D, 3 * H, generator=g) * 0.5).to(dev)
w = [(torch.rand(3 * H, H, generator=g) * 0.06 - 0.03).to(dev) for _ in range(2)]
b = [(torch.rand(3 * H, generator=g) * 0.06 - 0.03).to(dev) for _ in range(2)]
lens = torch.full((N,), T, dtype=torch.int32, device=dev)
h_all = torch.empty(T, N, D, H, device=dev)
gates = torch.empty(T, N, D, 4 * H, device=dev)
nbytes = _lib.size("ds2_gru_fwd_workspace_size", N, H, D)
ws = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
UB, KS, BT = (H + 15) // 16, (H + 3) // 4, (N + 15) // 16
al = lambda x: (x + 255) & ~255
off = al(D * UB * KS * 3 * 64 * 4) + al((D * BT + 1 + D * BT * 64) * 4)
for it in range(3):
    s0 = torch.cuda.Event(enable_timing=True); s1 = torch.cuda.Event(enable_timing=True)
    s0.record()
    _lib.call("ds2_gru_fwd", T, N, H, D, xproj.data_ptr(), w[0].data_ptr(), w[1].data_ptr(),
              b[0].data_ptr(), b[1].data_ptr(), lens.data_ptr(), h_all.data_ptr(),
              gates.data_ptr(), ws.data_ptr(), ws.numel(), ops._stream())
    s1.record()
    torch.cuda.synchronize()
    ms = s0.elapsed_time(s1)
    st = ws[off:off + 16 * 8].view(torch.int64).cpu().tolist()[:5]
    tot = sum(st)
    names = ["wait", "stage", "mfma+red", "pointwise", "arrive"]
    print(f"iter {it}: {ms:.3f} ms = {ms * 1e3 / T:.2f} us/step;  ticks/step: " +
          ", ".join(f"{nm} {v / T:.0f}" for nm, v in zip(names, st)) + f" total {tot / T:.0f}")

# backward timing (events only)
dy = torch.randn(T, N, H, device=dev)
dgx = torch.empty(T, N, D, 3 * H, device=dev)
dgh = torch.empty(T, N, D, 3 * H, device=dev)
wsb = torch.zeros(_lib.size("ds2_gru_bwd_workspace_size", N, H, D), dtype=torch.uint8, device=dev)
for it in range(3):
    s0 = torch.cuda.Event(enable_timing=True); s1 = torch.cuda.Event(enable_timing=True)
    s0.record()
    _lib.call("ds2_gru_bwd", T, N, H, D, dy.data_ptr(), 1, w[0].data_ptr(), w[1].data_ptr(),
              h_all.data_ptr(), gates.data_ptr(), lens.data_ptr(), dgx.data_ptr(), dgh.data_ptr(),
              wsb.data_ptr(), wsb.numel(), ops._stream())
    s1.record()
    torch.cuda.synchronize()
    ms = s0.elapsed_time(s1)
    print(f"bwd iter {it}: {ms:.3f} ms = {ms * 1e3 / T:.2f} us/step")
