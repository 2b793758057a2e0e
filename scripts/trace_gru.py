"""Diagnostic: per-workgroup timeline of the persistent GRU forward (DS2_GRU_STAMPS=2).

Every workgroup stamps s_memrealtime (10 ns ticks) at {step start, wait done, staged,
mfma+red done, arrived} for 16 steps; this prints the arrival skew inside each
(direction, batch tile) group, the latency from the group's last arrival to the
first / median / last consumer leaving its wait, and the phase lengths."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
os.environ["DS2_GRU_STAMPS"] = "2"
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ds2amd import _lib, ops  # noqa: E402

T, N, H, D = 501, 32, 800, 2
S0, NS = 100, 16
dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(0)
xproj = (torch.randn(T, N, D, 3 * H, generator=g) * 0.5).to(dev)
w = [(torch.rand(3 * H, H, generator=g) * 0.06 - 0.03).to(dev) for _ in range(2)]
b = [(torch.rand(3 * H, generator=g) * 0.06 - 0.03).to(dev) for _ in range(2)]
lens = torch.full((N,), T, dtype=torch.int32, device=dev)
h_all = torch.empty(T, N, D, H, device=dev)
gates = torch.empty(T, N, D, 4 * H, device=dev)
ws = torch.zeros(_lib.size("ds2_gru_fwd_workspace_size", N, H, D), dtype=torch.uint8, device=dev)
UB, KS, BT = (H + 15) // 16, (H + 3) // 4, (N + 15) // 16
al = lambda x: (x + 255) & ~255
off = al(D * UB * KS * 3 * 64 * 4) + al((D * BT + 1 + D * BT * 128) * 4)
P = UB * D
G = D * BT
# same-XCD groups (the default where they tile the XCDs; DS2_GRU_XCD=0 the interleaved layout)
XG = os.environ.get("DS2_GRU_XCD", "1")[:1] != "0" and 8 % G == 0 and UB % (8 // G) == 0
grid = 8 * (UB // (8 // G)) if XG else 8 * ((P + 7) // 8) * BT
# the XCD-local kernels (gru_xl.hip, the default at this shape; DS2_GRU_XL=0 the 16-unit ones):
# 32 units x 8 samples per workgroup, group = blocks with equal b % 8, grid 8 x H / 32
XL = os.environ.get("DS2_GRU_XL", "1")[:1] != "0" and H % 32 == 0 and D * ((N + 7) // 8) <= 8
if XL:
    grid = 8 * (H // 32)
for it in range(3):
    _lib.call("ds2_gru_fwd", T, N, H, D, xproj.data_ptr(), w[0].data_ptr(), w[1].data_ptr(),
              b[0].data_ptr(), b[1].data_ptr(), lens.data_ptr(), h_all.data_ptr(),
              gates.data_ptr(), None, ws.data_ptr(), ws.numel(), ops._stream())
    torch.cuda.synchronize()


# Floors of each phase from MI355X_MICROARCH.md (persistent-kernel price list, per-instruction
# table) for the fp16x3 kernels at this shape, printed beside the measured phases:
#  forward  -- sentinel ring (data-tagged: handoff-1to1, 1.0-1.4 us idle/loaded for <= 4 KB);
#              stage = UB 1-KB h tiles per workgroup per step at the handoff-payload rate
#              (62-70 GB/s per block cross-XCD, 104-122 same-XCD plain); MFMA = per wave 7
#              pairs x 3 gates x 3 v_mfma_f32_16x16x32_f16 (16 cycles/SIMD each), one wave/SIMD
#  backward -- flag hand-off (handoff-flag, drained sc1: 1.3 idle ... 1.7-1.9x handoff-1to1);
#              stage = UB records of 3.06 KB; MFMA = per wave 7 producers x (3 x 16 + 3 x 8)
#              cycles, two waves per SIMD
CLK_GHZ = 2.0
if XL:
    # stage: UBX tiles of 1 KB (forward) / records of 3.1 KB (backward) from the XCD's own L2
    # (handoff-payload same-XCD 104-122 GB/s per block); MFMA: per wave 7 producers x 12
    # v_mfma_f32_16x16x32_f16 (16 cycles each), one wave per SIMD
    UBX = H // 32
    FLOORS = {
        "forward": {"wait": (1.0, 1.4), "stage": (UBX * 1024 / 122e3, UBX * 1024 / 104e3),
                    "mfma": (7 * 12 * 16 / (CLK_GHZ * 1e3),) * 2},
        "backward": {"wait": (1.3, 2.5), "stage": (UBX * 3136 / 122e3, UBX * 3136 / 104e3),
                     "mfma": (7 * 12 * 16 / (CLK_GHZ * 1e3),) * 2},
    }
FLOORS_16 = {
    "forward": {"wait": (1.0, 1.4), "stage": (UB * 1024 / 122e3, UB * 1024 / 62e3),
                "mfma": (7 * 3 * 3 * 16 / (CLK_GHZ * 1e3),) * 2},
    "backward": {"wait": (1.3, 2.5), "stage": (UB * 3136 / 122e3, UB * 3136 / 62e3),
                 "mfma": (2 * 7 * (3 * 16 + 3 * 8) / (CLK_GHZ * 1e3),) * 2},
}
if not XL:
    FLOORS = FLOORS_16


def analyse(tr, label):
    print(f"--- {label}")
    fl = FLOORS.get(label)
    if fl is not None:
        print("floors (us, MI355X_MICROARCH): " + ", ".join(
            f"{k} {a:.2f}-{b:.2f}" for k, (a, b) in fl.items()))
    groups = {}
    for wg in range(grid):
        xcd, slot = wg & 7, wg >> 3
        if XL:
            if xcd < D * ((N + 7) // 8):
                groups.setdefault((xcd // ((N + 7) // 8), xcd % ((N + 7) // 8)), []).append(wg)
            continue
        if XG:
            q = xcd // (8 // G)
            groups.setdefault((q // BT, q % BT), []).append(wg)
            continue
        pair = xcd + 8 * (slot // BT)
        bt = slot % BT
        if pair >= P:
            continue
        d = pair // UB
        groups.setdefault((d, bt), []).append(wg)
    ticks_us = 0.01
    rows = []
    for s in range(NS - 1):
        for key, wgs in groups.items():
            arr = tr[s, wgs, 4].astype(np.float64)
            nxt_wait = tr[s + 1, wgs, 1].astype(np.float64)
            last = arr.max()
            rows.append(((arr.max() - arr.min()) * ticks_us, (np.sort(arr)[-2] - np.median(arr)) * ticks_us,
                         (nxt_wait.min() - last) * ticks_us, (np.median(nxt_wait) - last) * ticks_us,
                         (nxt_wait.max() - last) * ticks_us))
    r = np.array(rows)
    print("per group-step (us): arrival skew max-min %.2f | 2nd-last minus median arrival %.2f | "
          "last arrival -> first consumer %.2f, median %.2f, last %.2f" % tuple(r.mean(0)))
    ph = tr[1:NS - 1]
    valid = ph[..., 0] > 0
    def mean_phase(a, b_):
        return float(((ph[..., b_] - ph[..., a]) * ticks_us)[valid].mean())
    print("phases (us, mean over WGs/steps): wait %.2f, stage %.2f, mfma+red %.2f, pointwise+arrive %.2f"
          % (mean_phase(0, 1), mean_phase(1, 2), mean_phase(2, 3), mean_phase(3, 4)))
    v2 = tr[1:NS - 1, :, 0] > 0
    step_len = (tr[2:NS, :, 0] - tr[1:NS - 1, :, 0])[v2] * ticks_us
    print("step length (us): mean %.2f" % step_len.mean())
    # which WGs arrive last most often (systematic skew?)
    last_counts = {}
    for s in range(NS):
        for key, wgs in groups.items():
            wl = wgs[int(np.argmax(tr[s, wgs, 4]))]
            last_counts[wl] = last_counts.get(wl, 0) + 1
    top = sorted(last_counts.items(), key=lambda kv: -kv[1])[:8]
    print("most frequent last arrivers (wg: count, xcd):", [(k, v, k & 7) for k, v in top])
    # per-WG mean stage time by XCD
    st = ((ph[..., 2] - ph[..., 1]) * ticks_us)
    for x in range(8):
        cols = [wg for wg in range(grid) if (wg & 7) == x and any(wg in v for v in groups.values())]
        print(f"xcd {x}: stage {st[:, cols].mean():.2f} us, mfma {((ph[..., 3] - ph[..., 2]) * ticks_us)[:, cols].mean():.2f} us, wait {((ph[..., 1] - ph[..., 0]) * ticks_us)[:, cols].mean():.2f}")


def analyse_xl(tr, label):
    """The XCD-local kernels' per-wave stamps [step][block][wave][6]: step start, hand-off wait
    done, products done, io done, reduction barrier done, published."""
    print(f"--- {label} (XCD-local, per wave)")
    fl = FLOORS.get(label)
    if fl is not None:
        print("floors (us, MI355X_MICROARCH): " + ", ".join(
            f"{k} {a:.2f}-{b:.2f}" for k, (a, b) in fl.items()))
    G = D * ((N + 7) // 8)
    act = [b for b in range(grid) if (b & 7) < G]
    t = tr[:, act].astype(np.float64) * 0.01          # us
    ph = t[1:NS - 1]
    names = ["wait", "products", "io", "reduction barrier", "pointwise+publish"]
    for w in range(4):
        d_ = np.diff(ph[:, :, w, :], axis=-1)
        print(f"wave {w}: " + ", ".join(f"{nm} {d_[..., i].mean():.2f}" for i, nm in enumerate(names)))
    step = (t[2:NS, :, 0, 0] - t[1:NS - 1, :, 0, 0]).mean()
    print("step length (us): mean %.2f" % step)
    # per group: the last publish of step s -> each consumer's products done at s + 1
    rows = []
    for gq in range(G):
        bl = [i for i, b in enumerate(act) if (b & 7) == gq]
        for s_ in range(1, NS - 2):
            pub = t[s_, bl, 0, 5]
            nxt = t[s_ + 1, bl, :, 2].max(axis=1)
            rows.append(((pub.max() - pub.min()), (nxt.mean() - pub.max())))
    r = np.array(rows)
    print("publish skew within a group %.2f us; last publish -> consumers' products done %.2f us"
          % tuple(r.mean(0)))


if XL:
    analyse_xl(ws[off:off + NS * grid * 24 * 8].view(torch.int64).cpu().numpy().reshape(NS, grid, 4, 6),
               "forward")
else:
    analyse(ws[off:off + NS * grid * 5 * 8].view(torch.int64).cpu().numpy().reshape(NS, grid, 5),
            "forward")
dy = torch.randn(T, N, H, device=dev)
dgx = torch.empty(T, N, D, 3 * H, device=dev)
dgh = torch.empty(T, N, D, 3 * H, device=dev)
wsb = torch.zeros(_lib.size("ds2_gru_bwd_workspace_size", N, H, D), dtype=torch.uint8, device=dev)
for it in range(3):
    _lib.call("ds2_gru_bwd", T, N, H, D, dy.data_ptr(), 1, w[0].data_ptr(), w[1].data_ptr(),
              h_all.data_ptr(), gates.data_ptr(), lens.data_ptr(), dgx.data_ptr(), dgh.data_ptr(),
              None, wsb.data_ptr(), wsb.numel(), ops._stream())
    torch.cuda.synchronize()
KS3 = (3 * H + 3) // 4
offb = al(D * UB * KS3 * 64 * 4) + al(2 * N * D * H * 4) + al((D * BT + 1 + D * BT * 128) * 4)
if XL:
    analyse_xl(wsb[offb:offb + NS * grid * 24 * 8].view(torch.int64).cpu().numpy().reshape(NS, grid, 4, 6),
               "backward")
else:
    analyse(wsb[offb:offb + NS * grid * 5 * 8].view(torch.int64).cpu().numpy().reshape(NS, grid, 5),
            "backward")
