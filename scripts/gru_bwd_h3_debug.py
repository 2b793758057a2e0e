"""Debug probe: the fp16x3 GRU backward recurrence (gru_bwd_h3_kernel) against the bf16x6 one
(DS2_GRU_H3_BWD=0) on the same forward cache, through the C ABI: dgates_x / dgates_h, the
fused column maxima and the bias gradients, element by element (NaN positions, max error per
step), plus the hand-off status word.

usage: python scripts/gru_bwd_h3_debug.py [--n 19] [--t 9] [--h 400]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
from ds2amd import _lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=19)
    ap.add_argument("--t", type=int, default=9)
    ap.add_argument("--h", type=int, default=400)
    ap.add_argument("--nd", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda")
    n, t, h, nd = args.n, args.t, args.h, args.nd
    g = torch.Generator().manual_seed(1)
    xproj = (torch.randn(t, n, nd, 3 * h, generator=g) * 0.5).to(dev)
    w = [(torch.rand(3 * h, h, generator=g) * 0.2 - 0.1).to(dev) for _ in range(nd)]
    b = [(torch.rand(3 * h, generator=g) * 0.2 - 0.1).to(dev) for _ in range(nd)]
    lens = torch.tensor(sorted([max(1, t - i % t) for i in range(n)], reverse=True),
                        dtype=torch.int32, device=dev)
    h_all = torch.empty(t, n, nd, h, device=dev)
    gates = torch.empty(_lib.size("ds2_gru_cache_floats", t, n, h, nd), device=dev)
    st = ops.rnn_status_word(dev)
    ws = ops._ws(_lib.size("ds2_gru_fwd_workspace_size", n, h, nd), dev)
    _lib.call("ds2_gru_fwd", t, n, h, nd, xproj.data_ptr(), w[0].data_ptr(),
              w[1].data_ptr() if nd == 2 else None, b[0].data_ptr(),
              b[1].data_ptr() if nd == 2 else None, lens.data_ptr(), h_all.data_ptr(),
              gates.data_ptr(), st.data_ptr(), ws.data_ptr(), ws.numel(), ops._stream())
    dy = torch.randn(t, n, nd, h, generator=g).to(dev)
    res = {}
    for mode in ("1", "0"):
        os.environ["DS2_GRU_H3_BWD"] = mode
        dgx = torch.full((t, n, nd, 3 * h), 7.0, device=dev)
        dgh = torch.full((t, n, nd, 3 * h), 7.0, device=dev)
        db = [torch.zeros(3 * h, device=dev) for _ in range(4)]
        camax = torch.zeros(2 * nd * 3 * h, dtype=torch.int32, device=dev)
        ws = ops._ws(_lib.size("ds2_gru_bwd_workspace_size", n, h, nd), dev)
        st.zero_()
        _lib.call("ds2_gru_bwd_bias_amax", t, n, h, nd, dy.data_ptr(), nd, w[0].data_ptr(),
                  w[1].data_ptr() if nd == 2 else None, h_all.data_ptr(), gates.data_ptr(),
                  lens.data_ptr(), dgx.data_ptr(), dgh.data_ptr(), db[0].data_ptr(),
                  db[1].data_ptr(), db[2].data_ptr() if nd == 2 else None,
                  db[3].data_ptr() if nd == 2 else None, camax.data_ptr(), st.data_ptr(),
                  ws.data_ptr(), ws.numel(), ops._stream())
        torch.cuda.synchronize()
        res[mode] = (dgx.cpu(), dgh.cpu(), [x.cpu() for x in db], camax.cpu(), int(st.item()))
        print(f"mode H3_BWD={mode}: status {int(st.item())}, dgx NaN {int(dgx.isnan().sum())}, "
              f"dgh NaN {int(dgh.isnan().sum())}, dgx==7 {int((dgx == 7).sum())}", flush=True)
    a, r = res["1"], res["0"]
    for name, x, y in (("dgx", a[0], r[0]), ("dgh", a[1], r[1])):
        for tt in range(t):
            for d in range(nd):
                e = (x[tt, :, d] - y[tt, :, d]).abs()
                print(f"{name} t={tt} d={d}: max err {e.max().item():.3e} (ref max "
                      f"{y[tt, :, d].abs().max().item():.3e}) nan rows "
                      f"{[int(i) for i in torch.nonzero(x[tt, :, d].isnan().any(1)).flatten()][:8]}",
                      flush=True)
    for i in range(4):
        e = (a[2][i] - r[2][i]).abs().max().item()
        print(f"db[{i}] max err {e:.3e} (ref max {r[2][i].abs().max().item():.3e})")
    ref_cm = torch.cat([r[0].abs().view(-1, nd * 3 * h).amax(0), r[1].abs().view(-1, nd * 3 * h).amax(0)])
    got_cm = a[3].view(torch.float32)
    rel = ((got_cm - ref_cm).abs() / ref_cm.clamp_min(1e-30))
    print(f"camax: max rel diff {rel.max().item():.3e}; below ref by > 1e-3 at "
          f"{int((got_cm < ref_cm * (1 - 1e-3)).sum())} of {ref_cm.numel()} columns")


if __name__ == "__main__":
    main()
