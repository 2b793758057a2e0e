"""Debug probe for the fp16x3 GEMM's operand scales: ds2_amax against torch, and the GEMM with
the library's own scales vs scales supplied from torch (ds2_sgemm_amax_ws), on step shapes with
rows / columns spread over 12 decades."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch
from ds2amd import _lib, ops
dev = torch.device("cuda")
os.environ["DS2_GEMM_H3"] = "1"
torch.manual_seed(1)


def bits(v):
    return v.float().contiguous().view(torch.int32)


for name, ta, tb, m, n, k in (("dX NN", 0, 0, 16032, 800, 4800), ("dW TN", 1, 0, 4800, 800, 16032),
                              ("small NN", 0, 0, 512, 320, 1024), ("xproj NT", 0, 1, 16032, 4800, 800)):
    a = torch.randn((k, m) if ta else (m, k), device=dev)
    b = torch.randn((n, k) if tb else (k, n), device=dev)
    sa = torch.pow(10.0, torch.empty(m, device=dev).uniform_(-6, 6))
    sb = torch.pow(10.0, torch.empty(n, device=dev).uniform_(-6, 6))
    a = a * sa[None, :] if ta else a * sa[:, None]
    b = b * sb[:, None] if tb else b * sb[None, :]
    at = a.t() if ta else a
    bt = b.t() if tb else b
    ref = torch.mm(at.double(), bt.double())
    am_a = at.abs().amax(1)
    am_b = bt.abs().amax(0)
    # ds2_amax on the stored matrices
    ra = torch.zeros(a.shape[0], dtype=torch.int32, device=dev)
    ca = torch.zeros(a.shape[1], dtype=torch.int32, device=dev)
    _lib.call("ds2_amax", a.data_ptr(), a.shape[0], a.shape[1], a.shape[1], ra.data_ptr(), ca.data_ptr(), ops._stream())
    rb = torch.zeros(b.shape[0], dtype=torch.int32, device=dev)
    cb = torch.zeros(b.shape[1], dtype=torch.int32, device=dev)
    _lib.call("ds2_amax", b.data_ptr(), b.shape[0], b.shape[1], b.shape[1], rb.data_ptr(), cb.data_ptr(), ops._stream())
    torch.cuda.synchronize()
    ok_ra = torch.equal(ra, bits(a.abs().amax(1)))
    ok_ca = torch.equal(ca, bits(a.abs().amax(0)))
    ok_rb = torch.equal(rb, bits(b.abs().amax(1)))
    ok_cb = torch.equal(cb, bits(b.abs().amax(0)))
    c = torch.empty(m, n, device=dev)
    nbytes = _lib.size("ds2_sgemm_workspace_size", m, n, k, 1)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    res = []
    for label, pa, pb in (("own", None, None), ("torch", bits(am_a), bits(am_b))):
        _lib.call("ds2_sgemm_amax_ws", ta, tb, m, n, k, 1.0, a.data_ptr(), a.shape[1], b.data_ptr(),
                  b.shape[1], 0.0, c.data_ptr(), n, None, None if pa is None else pa.data_ptr(),
                  None if pb is None else pb.data_ptr(), ws.data_ptr(), nbytes, ops._stream())
        torch.cuda.synchronize()
        nanr = torch.isnan(c).any(1).nonzero().flatten()
        nanc = torch.isnan(c).any(0).nonzero().flatten()
        err = ((c.double() - ref).abs() / torch.mm(at.double().abs(), bt.double().abs())).max().item()
        res.append(f"{label}: nan rows {nanr.numel()} cols {nanc.numel()} first r {nanr[:3].tolist()} c {nanc[:3].tolist()} comp {err:.1e}")
    print(f"{name}: amax a rows {ok_ra} cols {ok_ca} b rows {ok_rb} cols {ok_cb} | " + " | ".join(res), flush=True)
