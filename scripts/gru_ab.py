"""A/B timing of the GRU recurrence variants at the bench shape (T=501, N=32, H=800,
bidirectional), alternating in one process: the bf16x6 kernels vs the fp32-MFMA ones, the
same-XCD groups vs the interleaved layout, and poll-knob sweeps (DS2_RNN_TUNE) -- selected
through the environment switches the library reads at every call."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
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
dy = torch.randn(T, N, H, generator=g).to(dev)
dgx = torch.empty(T, N, D, 3 * H, device=dev)
dgh = torch.empty(T, N, D, 3 * H, device=dev)
wsf = torch.zeros(_lib.size("ds2_gru_fwd_workspace_size", N, H, D), dtype=torch.uint8, device=dev)
wsb = torch.zeros(_lib.size("ds2_gru_bwd_workspace_size", N, H, D), dtype=torch.uint8, device=dev)


def fwd():
    _lib.call("ds2_gru_fwd", T, N, H, D, xproj.data_ptr(), w[0].data_ptr(), w[1].data_ptr(),
              b[0].data_ptr(), b[1].data_ptr(), lens.data_ptr(), h_all.data_ptr(),
              gates.data_ptr(), None, wsf.data_ptr(), wsf.numel(), ops._stream())


def bwd():
    _lib.call("ds2_gru_bwd", T, N, H, D, dy.data_ptr(), 1, w[0].data_ptr(), w[1].data_ptr(),
              h_all.data_ptr(), gates.data_ptr(), lens.data_ptr(), dgx.data_ptr(),
              dgh.data_ptr(), None, wsb.data_ptr(), wsb.numel(), ops._stream())


def xl_modes():
    """The XCD-local kernels' per-group mode words (1 LOCAL, 2 GLOBAL, 3 mixed) of the last
    forward and backward launches, read from the workspaces' counter area."""
    if os.environ.get("DS2_GRU_XL", "1")[:1] == "0":
        return ""
    al = lambda x: (x + 255) & ~255
    UB, BT = (H + 15) // 16, (N + 15) // 16
    cf = al(D * UB * ((H + 3) // 4) * 3 * 64 * 4)
    cb = al(D * UB * ((3 * H + 3) // 4) * 64 * 4) + al(2 * N * D * H * 4)
    out = []
    for ws, c in ((wsf, cf), (wsb, cb)):
        words = ws[c:c + 4 * (D * BT + 1 + 520)].view(torch.int32).cpu()
        out.append(words[D * BT + 1 + 512: D * BT + 1 + 520].tolist())
    return f"  modes fwd {out[0]} bwd {out[1]}"


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


variants = {"x6": {"DS2_GRU_X6": "1", "DS2_RNN_TUNE": ""},
            "f32": {"DS2_GRU_X6": "0", "DS2_RNN_TUNE": ""}}
if len(sys.argv) > 1 and sys.argv[1] == "xcd":
    # the same-XCD groups vs the interleaved layout (DS2_GRU_XCD, read at every call)
    variants = {f"xcd{v}": {"DS2_GRU_X6": "1", "DS2_GRU_XCD": v} for v in ("1", "0")}
if len(sys.argv) > 1 and sys.argv[1] == "ftune":
    # the sentinel forward's first-poll delay / re-poll sleep (s_sleep units)
    variants = {f"fwd-tune-{t}": {"DS2_GRU_X6": "1", "DS2_RNN_TUNE": t}
                for t in ("1,10,14", "1,0,14", "1,4,14", "1,7,14", "1,14,14", "0,7,14", "2,7,14")}
if len(sys.argv) > 1 and sys.argv[1] == "flagpoll":
    # s_sleep(1) units between the flag hand-off's polls (the pre-split backward's wait)
    variants = {f"bwd-poll-{t}": {"DS2_GRU_X6": "1", "DS2_RNN_TUNE": t}
                for t in ("1,10,14,1", "1,10,14,0", "1,10,14,2", "1,10,14,4")}
if len(sys.argv) > 1 and sys.argv[1] == "flagpipe":
    # the flag hand-off with a second poll in flight, issued G s_sleep(1) units after the first
    # (0: one poll at a time)
    variants = {f"bwd-pipe-{g}": {"DS2_RNN_TUNE": f"1,10,14,1,{g}"} for g in ("0", "4", "8", "14", "20")}
if len(sys.argv) > 1 and sys.argv[1] == "flagdelay":
    # s_sleep(1) units before the backward's first flag poll of a step ([5]) and between polls ([3])
    variants = {f"bwd-flagdelay-{t}": {"DS2_RNN_TUNE": f"1,10,14,{t}"}
                for t in ("1,0,0", "1,0,8", "1,0,16", "1,0,24", "2,0,16", "4,0,16")}
if len(sys.argv) > 1 and sys.argv[1] == "xl":
    # the XCD-local kernels (gru_xl.hip) LOCAL (plain stores, default), forced GLOBAL (sc1), and
    # the 16-unit fp16x3 kernels they replace
    variants = {"xl-local": {"DS2_GRU_XL": "1", "DS2_RNN_TUNE": ""},
                "xl-global": {"DS2_GRU_XL": "2", "DS2_RNN_TUNE": ""},
                "16unit": {"DS2_GRU_XL": "0", "DS2_RNN_TUNE": ""}}
if len(sys.argv) > 1 and sys.argv[1] == "xlrepoll":
    # the XCD-local forward: tiles re-loaded per stale pass (DS2_RNN_TUNE [6]) x first-poll delay
    variants = {f"xl-rp-{t}": {"DS2_GRU_XL": "1", "DS2_RNN_TUNE": t}
                for t in ("1,7,14,1,0,0,8,7", "1,7,14,1,0,0,1,0", "1,7,14,1,0,0,2,0",
                          "1,7,14,1,0,0,1,3", "0,7,14,1,0,0,1,0", "1,7,14,1,0,0,8,0")}
if len(sys.argv) > 1 and sys.argv[1] == "xlonly":
    variants = {"xl-local": {"DS2_GRU_XL": "1", "DS2_RNN_TUNE": ""}}
if len(sys.argv) > 1 and sys.argv[1] == "xltune":
    # the XCD-local forward's first-poll delay / re-poll sleep (s_sleep units)
    variants = {f"xl-tune-{t}": {"DS2_GRU_XL": "1", "DS2_RNN_TUNE": t}
                for t in ("1,7,14", "1,0,14", "1,3,14", "0,0,14", "0,3,14", "2,3,14")}
rounds = int(os.environ.get("AB_ROUNDS", "3"))
variants = {f"{k}#{r}": v for r in range(rounds) for k, v in variants.items()}
ref = None
for name, env in variants.items():
    os.environ.update(env)
    tf = timed(fwd)
    out_h = h_all.clone()
    tb = timed(bwd)
    out_g = dgx.clone()
    if ref is None:
        ref = (out_h, out_g)
    dh = (out_h - ref[0]).abs().max().item()
    dg = (out_g - ref[1]).abs().max().item() / max(ref[1].abs().max().item(), 1e-30)
    print(f"{name:12s} fwd {tf * 1e3:8.1f} us ({tf * 1e3 / T:5.2f}/step)  bwd {tb * 1e3:8.1f} us "
          f"({tb * 1e3 / T:5.2f}/step)  max|dh| {dh:.2e} rel|ddgx| {dg:.2e}{xl_modes()}", flush=True)
