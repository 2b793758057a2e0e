"""GPU: every HIP kernel against a CPU reference of the same op (fp64 where cheap).

Tolerances (fp32 kernels): relative to the magnitude of the result, 1e-5..1e-4;
integer/index outputs (greedy decode, lengths) bit-exact.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from ds2amd import ops, _lib
from oracle import ds2_oracle as orc

pytestmark = pytest.mark.gpu


def _close(got, ref, rel=1e-5, name=""):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    scale = max(ref.abs().max().item(), 1e-30)
    err = (got - ref).abs().max().item()
    assert err <= rel * scale, f"{name}: max err {err:.3e} > {rel:.1e} * {scale:.3e}"


# ---------------------------------------------------------------------------- GEMM
def _gemm_mode(monkeypatch, mode):
    """x6: the bf16x6 kernel; h3: the fp16x3 kernel (DS2_GEMM_H3=1); fp32: DS2_GEMM_X6=0."""
    monkeypatch.setenv("DS2_GEMM_X6", "0" if mode.startswith("fp32") or mode == "unaligned"
                       else "1")
    monkeypatch.setenv("DS2_GEMM_H3", "1" if mode.startswith("h3") else "0")


@pytest.mark.parametrize("x6", ["1", "0", "h3"])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("m,n,k", [(1, 1, 1), (37, 53, 29), (128, 128, 16), (300, 257, 513),
                                   (515, 2400, 132), (257, 300, 5000),   # split-K path
                                   (300, 256, 516), (260, 132, 1000),    # float4 staging, K % 32 != 0
                                   (300, 260, 1024)])                    # K % 32 == 0
def test_sgemm(dev, ta, tb, m, n, k, x6, monkeypatch):
    """ds2_sgemm_ws vs fp64 at 1e-5: the bf16x6 kernel (256 x 160 tiles for N >= 256,
    256 x 128 below; its 16x16x32 form where every stage lies inside K, the 32x32x16 form for
    a K tail), the fp16x3 kernel ("h3", the same tiles on v_mfma_f32_16x16x32_f16 where every
    stage lies inside K, else the bf16x6 kernel) and the fp32-MFMA kernels (DS2_GEMM_X6=0)."""
    _gemm_mode(monkeypatch, {"1": "x6", "0": "fp32", "h3": "h3"}[x6])
    g = torch.Generator().manual_seed(m * 7 + n * 3 + k)
    a = torch.randn(k, m, generator=g) if ta else torch.randn(m, k, generator=g)
    b = torch.randn(n, k, generator=g) if tb else torch.randn(k, n, generator=g)
    c0 = torch.randn(m, n, generator=g)
    bias = torch.randn(n, generator=g)
    ref = 0.5 * ((a.t() if ta else a).double() @ (b.t() if tb else b).double()) \
        + 0.25 * c0.double() + bias.double()
    ad, bd, cd = a.to(dev), b.to(dev), c0.to(dev).clone()
    ops.sgemm(ad, bd, cd, m=m, n=n, k=k, trans_a=bool(ta), trans_b=bool(tb),
              lda=ad.shape[1], ldb=bd.shape[1], ldc=n, alpha=0.5, beta=0.25, bias=bias.to(dev))
    torch.cuda.synchronize()
    _close(cd, ref, 1e-5, "sgemm")


@pytest.mark.parametrize("mode", ["x6", "x6-narrow", "x6-ktail", "x6-ktail-narrow", "fp32",
                                  "fp32-narrow", "unaligned", "h3", "h3-narrow"])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_sgemm_full_rounds_plus_split_tail(dev, ta, tb, mode, monkeypatch):
    """Whole rounds of resident workgroups + a tail whose K range is split (one launch) and
    reduced in a fixed order; alpha/beta/bias applied once.  bf16x6 kernel: 256 x 160 tiles
    (N >= 256) and 256 x 128 ("-narrow": N < 256); fp32 kernels (DS2_GEMM_X6=0): BK = 64 /
    16x16x4 with the plan's tile width, and ("unaligned": A one float off 16-B alignment)
    the BK = 16 / 32x32x2 kernel."""
    _gemm_mode(monkeypatch, mode)
    # K % 32 == 0: the 16x16x32 form; "-ktail" (K % 32 == 4): the 32x32x16 form with k checks
    m, k = 128 * 29, 2084 if "ktail" in mode else 2080
    n = 200 if mode.endswith("narrow") else 128 * 27 + 52
    g = torch.Generator().manual_seed(5)
    a = torch.randn(k, m, generator=g) if ta else torch.randn(m, k, generator=g)
    b = torch.randn(n, k, generator=g) if tb else torch.randn(k, n, generator=g)
    c0 = torch.randn(m, n, generator=g)
    bias = torch.randn(n, generator=g)
    ref = 0.5 * ((a.t() if ta else a).double() @ (b.t() if tb else b).double()) \
        + 0.25 * c0.double() + bias.double()
    ad, bd, cd = a.to(dev), b.to(dev), c0.to(dev).clone()
    a_off, lda = 0, ad.shape[1]
    if mode == "unaligned":
        buf = torch.empty(ad.numel() + 1, device=dev)
        buf[1:].copy_(ad.reshape(-1))
        ad, a_off = buf, 1
    ops.sgemm(ad, bd, cd, m=m, n=n, k=k, trans_a=bool(ta), trans_b=bool(tb),
              lda=lda, ldb=bd.shape[1], ldc=n, alpha=0.5, beta=0.25, bias=bias.to(dev),
              a_off=a_off)
    torch.cuda.synchronize()
    _close(cd, ref, 1e-5, "sgemm main+tail")


@pytest.mark.parametrize("ta,tb,m,n,k", [(0, 1, 2048, 2400, 800), (0, 0, 2048, 800, 2400),
                                         (1, 0, 2400, 800, 4096), (1, 0, 2400, 1312, 4096)])
def test_sgemm_x6_is_fp32_accurate(dev, ta, tb, m, n, k, monkeypatch):
    """The bf16x6 kernel's error against fp64 is of the fp32-MFMA kernel's order on the
    step's GEMM shapes (rows cut to keep the test short; measured 0.6-1.8x of it, both
    ~1e-6 of max |C|): an fp32 GEMM, not a reduced-precision one (a plain bf16 product
    is ~1e-3 off here)."""
    g = torch.Generator().manual_seed(m + n + k)
    a = (torch.randn(k, m, generator=g) if ta else torch.randn(m, k, generator=g)).to(dev)
    b = (torch.randn(n, k, generator=g) if tb else torch.randn(k, n, generator=g)).to(dev)
    ref = (a.t() if ta else a).double() @ (b.t() if tb else b).double()
    scale = ref.abs().max().item()
    errs = {}
    for mode in ("x6", "fp32", "h3"):
        _gemm_mode(monkeypatch, mode)
        c = torch.empty(m, n, device=dev)
        ops.sgemm(a, b, c, m=m, n=n, k=k, trans_a=bool(ta), trans_b=bool(tb), lda=a.shape[1],
                  ldb=b.shape[1], ldc=n)
        errs[mode] = (c.double() - ref).abs().max().item() / scale
    assert errs["x6"] <= 2.5 * errs["fp32"] and errs["x6"] < 5e-6, errs
    assert errs["h3"] <= 2.5 * errs["fp32"] and errs["h3"] < 5e-6, errs


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_sgemm_h3_rows_over_twelve_decades(dev, ta, tb, monkeypatch):
    """The fp16x3 kernel's per-row scales: rows of op(A) and columns of op(B) scaled by
    10^U(-6, 6), so one unscaled fp16 range could not hold them.  Componentwise error
    max |C - C64| / (|A| |B|) (the form of the fp32 GEMM error bound) within 2.5x of the
    fp32-MFMA kernel's and < 1e-6; the caller-supplied scales (ds2_sgemm_amax_ws, from
    ds2_amax) give the same bits as the kernel's own pre-pass."""
    m, n, k = 600, 416, 1088
    g = torch.Generator().manual_seed(17 + 2 * ta + tb)
    a = torch.randn(k, m, generator=g) if ta else torch.randn(m, k, generator=g)
    b = torch.randn(n, k, generator=g) if tb else torch.randn(k, n, generator=g)
    sa = torch.pow(10.0, torch.rand(m, generator=g) * 12 - 6)
    sb = torch.pow(10.0, torch.rand(n, generator=g) * 12 - 6)
    a = (a * sa[None, :] if ta else a * sa[:, None]).to(dev)
    b = (b * sb[:, None] if tb else b * sb[None, :]).to(dev)
    at, bt = (a.t() if ta else a).double(), (b.t() if tb else b).double()
    ref = at @ bt
    bound = at.abs() @ bt.abs()
    comp = {}
    outs = {}
    for mode in ("fp32", "h3"):
        _gemm_mode(monkeypatch, mode)
        c = torch.empty(m, n, device=dev)
        ops.sgemm(a, b, c, m=m, n=n, k=k, trans_a=bool(ta), trans_b=bool(tb), lda=a.shape[1],
                  ldb=b.shape[1], ldc=n)
        torch.cuda.synchronize()
        assert torch.isfinite(c).all().item(), mode
        comp[mode] = ((c.double() - ref).abs() / bound).max().item()
        outs[mode] = c
    assert comp["h3"] <= 2.5 * comp["fp32"] and comp["h3"] < 1e-6, comp
    # the same with the scales computed by ds2_amax and handed in
    am_a = torch.zeros(a.shape[0], dtype=torch.int32, device=dev)
    am_b = torch.zeros(b.shape[0] if tb else b.shape[1], dtype=torch.int32, device=dev)
    ca = torch.zeros(a.shape[1], dtype=torch.int32, device=dev)
    if ta:
        _lib.call("ds2_amax", a.data_ptr(), k, m, m, None, ca.data_ptr(), ops._stream())
        am_a = ca
    else:
        _lib.call("ds2_amax", a.data_ptr(), m, k, k, am_a.data_ptr(), None, ops._stream())
    if tb:
        _lib.call("ds2_amax", b.data_ptr(), n, k, k, am_b.data_ptr(), None, ops._stream())
    else:
        _lib.call("ds2_amax", b.data_ptr(), k, n, n, None, am_b.data_ptr(), ops._stream())
    c2 = torch.empty(m, n, device=dev)
    ops.sgemm(a, b, c2, m=m, n=n, k=k, trans_a=bool(ta), trans_b=bool(tb), lda=a.shape[1],
              ldb=b.shape[1], ldc=n, a_amax=am_a, b_amax=am_b)
    torch.cuda.synchronize()
    assert torch.equal(c2, outs["h3"])


@pytest.mark.parametrize("rows,cols", [(1, 4), (37, 52), (4800, 800), (5, 2048), (16032, 4800), (16032, 2400),
                                       (300, 4100)])
def test_amax_rows_and_cols(dev, rows, cols):
    """ds2_amax: row and column maxima of |x| in one pass, bit-exact against torch (float bits;
    a NaN is skipped, an inf kept) -- one wave per row up to 2048 columns (the stacked W_ih the
    input projection and dX share), row-block tiles beyond -- and rows alone through the
    one-wave-per-row kernel too."""
    g = torch.Generator().manual_seed(rows + cols)
    x = torch.randn(rows, cols + 8, generator=g) * torch.pow(10.0, torch.rand(rows, 1, generator=g) * 8 - 4)
    if rows > 3 and cols > 3:
        x[1, 2] = float('nan')
        x[2, 3] = float('-inf')
    x = x.to(dev)
    view = x[:, :cols]
    ref = view.abs().nan_to_num(nan=0.0, posinf=float('inf'))
    r = torch.zeros(rows, dtype=torch.int32, device=dev)
    c = torch.zeros(cols, dtype=torch.int32, device=dev)
    _lib.call("ds2_amax", x.data_ptr(), rows, cols, cols + 8, r.data_ptr(), c.data_ptr(),
              ops._stream())
    torch.cuda.synchronize()
    assert torch.equal(r, ref.amax(1).contiguous().view(torch.int32))
    assert torch.equal(c, ref.amax(0).contiguous().view(torch.int32))
    r2 = torch.zeros(rows, dtype=torch.int32, device=dev)
    _lib.call("ds2_amax", x.data_ptr(), rows, cols, cols + 8, r2.data_ptr(), None, ops._stream())
    torch.cuda.synchronize()
    assert torch.equal(r2, r)


@pytest.mark.parametrize("ta,tb", [(0, 1), (1, 0)])
def test_sgemm_x6_nonfinite_operands(dev, ta, tb, monkeypatch):
    """Bad-data semantics of the bf16x6 split: an inf operand splits into
    hi = inf and NaN residual terms, so its products are NaN where fp32 gives +-inf (or
    NaN).  Pinned here: the set of non-finite outputs equals the fp32-MFMA kernel's
    (DS2_GEMM_X6=0) and every finite output still matches it -- the NaN guard of the step
    sees the same rows either way.  (Finite values within 0.4 % of FLT_MAX round to a
    bf16 inf and are the one case where a finite fp32 result turns non-finite.)"""
    m, n, k = 256, 160, 96
    g = torch.Generator().manual_seed(11)
    a = torch.randn(k, m, generator=g) if ta else torch.randn(m, k, generator=g)
    b = torch.randn(n, k, generator=g) if tb else torch.randn(k, n, generator=g)
    if ta:
        a[5, 7] = float('inf'); a[9, 100] = float('-inf'); a[3, 40] = float('nan')
    else:
        a[7, 5] = float('inf'); a[100, 9] = float('-inf'); a[40, 3] = float('nan')
    b[2, 3] = float('inf')
    a, b = a.to(dev), b.to(dev)
    out = {}
    for mode in ("x6", "fp32", "h3"):
        _gemm_mode(monkeypatch, mode)
        c = torch.empty(m, n, device=dev)
        ops.sgemm(a, b, c, m=m, n=n, k=k, trans_a=bool(ta), trans_b=bool(tb), lda=a.shape[1],
                  ldb=b.shape[1], ldc=n)
        out[mode] = c.cpu()
    bad0 = ~torch.isfinite(out["fp32"])
    assert bad0.any()
    fin = ~bad0
    for mode in ("x6", "h3"):   # the fp16x3 split: an inf row keeps scale 1, inf - inf = NaN
        assert torch.equal(~torch.isfinite(out[mode]), bad0), mode
        assert (out[mode][fin] - out["fp32"][fin]).abs().max().item() <= \
            1e-4 * out["fp32"][fin].abs().max().item(), mode


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("m,n,k", [(4, 4, 4), (36, 52, 28), (128, 128, 64), (300, 256, 516),
                                   (516, 2400, 132), (256, 300, 5000),      # split-K tail
                                   (128 * 29, 128 * 27 + 52, 2080)])       # rounds + tail
def test_sgemm_bf16(dev, ta, tb, m, n, k):
    """bf16-operand GEMM (BASELINE cfg4): operands rounded to bf16 (nearest even) on the
    way in, exact products, fp32 accumulation.  Reference: the same bf16 roundings done by
    torch on the host, multiplied in fp64 -- so only the fp32 summation differs (1e-5)."""
    g = torch.Generator().manual_seed(m * 7 + n * 3 + k + 1)
    a = torch.randn(k, m, generator=g) if ta else torch.randn(m, k, generator=g)
    b = torch.randn(n, k, generator=g) if tb else torch.randn(k, n, generator=g)
    c0 = torch.randn(m, n, generator=g)
    bias = torch.randn(n, generator=g)
    rb = lambda t: t.to(torch.bfloat16).double()
    ref = 0.5 * ((rb(a).t() if ta else rb(a)) @ (rb(b).t() if tb else rb(b))) \
        + 0.25 * c0.double() + bias.double()
    ad, bd, cd = a.to(dev), b.to(dev), c0.to(dev).clone()
    ops.sgemm(ad, bd, cd, m=m, n=n, k=k, trans_a=bool(ta), trans_b=bool(tb),
              lda=ad.shape[1], ldb=bd.shape[1], ldc=n, alpha=0.5, beta=0.25, bias=bias.to(dev),
              bf16=True)
    torch.cuda.synchronize()
    _close(cd, ref, 1e-5, "sgemm bf16")
    # and it is a bf16 product: far from the fp32 one at this scale
    full = 0.5 * ((a.t() if ta else a).double() @ (b.t() if tb else b).double()) \
        + 0.25 * c0.double() + bias.double()
    if k >= 28:
        assert (cd.double().cpu() - full).abs().max() > 1e-4 * full.abs().max()


@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (300, 200, 136), (1000, 520, 1024),
                                   (513, 777, 4104), (2048, 4096, 1312),
                                   (4096, 1024, 32064 // 4), (64, 1024, 32064)])
def test_bgemm_nt(dev, m, n, k):
    """ds2_bgemm_nt (bf16 operands in HBM, the 256 x 256 LDS-DMA ping-pong kernel): partial
    tiles in M and N, K not a multiple of 64 (the masked last K-tile), whole rounds plus a
    split-K tail, one tile row with deep K.  Reference: the same bf16 values multiplied in
    fp64 -- only the fp32 summation order differs (1e-5).  ds2_cvt_bf16 (RNE) equals torch's
    bf16 rounding bit for bit, plain and transposed."""
    g = torch.Generator().manual_seed(m + n + k)
    a32 = torch.randn(m, k, generator=g).to(dev)
    b32 = torch.randn(k, n, generator=g).to(dev)          # n-contiguous: the transposing copy
    c0 = torch.randn(m, n, generator=g).to(dev)
    bias = torch.randn(n, generator=g).to(dev)
    a = ops.to_bf16(a32)
    bt = ops.to_bf16(b32, transpose=True)                  # [n, k]
    assert torch.equal(a, a32.to(torch.bfloat16))
    assert torch.equal(bt, b32.t().contiguous().to(torch.bfloat16))
    c = c0.clone()
    ops.bgemm_nt(a, bt, c, alpha=0.5, beta=0.25, bias=bias)
    torch.cuda.synchronize()
    ref = 0.5 * (a.double() @ bt.double().t()) + 0.25 * c0.double() + bias.double()
    _close(c, ref, 1e-5, "bgemm_nt")


@pytest.mark.parametrize("rows,cols", [(37, 53), (64, 64), (130, 96), (96, 130), (100, 8),
                                       (1000, 1312), (65, 4100)])
@pytest.mark.parametrize("transpose", [False, True])
def test_cvt_bf16(dev, rows, cols, transpose):
    """ds2_cvt_bf16 equals torch's bf16 rounding bit for bit on the 16-B vector paths (row
    runs / LDS-transposed 8-row runs) and the element paths (strides not multiples of 4 / 8),
    with partial 64 x 64 tiles and run tails in both directions."""
    g = torch.Generator().manual_seed(rows * 7 + cols)
    x = torch.randn(rows, cols, generator=g).to(dev)
    y = ops.to_bf16(x, transpose=transpose)
    ref = (x.t().contiguous() if transpose else x).to(torch.bfloat16)
    assert torch.equal(y, ref)


def test_sgemm_bf16_rejects_unaligned(dev):
    a = torch.randn(8, 6, device=dev)
    b = torch.randn(6, 8, device=dev)
    c = torch.empty(8, 8, device=dev)
    with pytest.raises(_lib.Ds2Error):
        ops.sgemm(a, b, c, m=8, n=8, k=6, lda=6, ldb=8, ldc=8, bf16=True)


# ---------------------------------------------------------------------------- conv
CONVS = [  # (n, ci, h, w, co, kh, kw, sh, sw, ph, pw)
    (2, 1, 161, 37, 32, 41, 11, 2, 2, 20, 5),
    # one input channel -> LDS-patch conv1 kernel: two column tiles, edge rows, fewer
    # output channels, other strides / taps
    (2, 1, 161, 300, 32, 41, 11, 2, 2, 20, 5),
    (2, 1, 33, 260, 20, 7, 5, 3, 2, 3, 2),
    (2, 1, 20, 150, 16, 5, 4, 1, 1, 2, 1),
    (2, 32, 81, 23, 32, 21, 11, 2, 1, 10, 5),
    (3, 3, 17, 300, 40, 5, 3, 1, 2, 2, 1),
    # width stride 1 -> LDS-patch direct kernels (several column tiles, two output-channel
    # blocks, 3 stride classes in dgrad, odd tap counts, edge rows / columns)
    (2, 32, 81, 200, 32, 21, 11, 2, 1, 10, 5),
    # conv2's kernel columns with fewer channels and tap rows (bf16x6 wgrad: partial
    # channel blocks, idle tap-row waves, one output row per split)
    (3, 5, 30, 70, 20, 7, 11, 1, 1, 3, 5),
    (3, 5, 19, 140, 40, 3, 3, 1, 1, 1, 1),
    (2, 4, 30, 50, 8, 7, 5, 3, 1, 3, 2),
    (1, 2, 9, 7, 3, 4, 2, 2, 1, 3, 0),
]


def _conv_mode(monkeypatch, mode):
    """h3: the default (fp16x3 conv2-shaped fwd / dgrad and sliding-window wgrad, bf16x6
    elsewhere); x6: bf16x6 (DS2_CONV_H3=0, DS2_CONV_H3W=0); fp32: the fp32 LDS-patch /
    implicit-GEMM kernels (DS2_CONV_X6=0)."""
    monkeypatch.setenv("DS2_CONV_X6", "0" if mode == "fp32" else "1")
    monkeypatch.setenv("DS2_CONV_H3", "1" if mode == "h3" else "0")
    monkeypatch.setenv("DS2_CONV_H3W", "1" if mode == "h3" else "0")


@pytest.mark.parametrize("mode", ["h3", "x6", "fp32"])
@pytest.mark.parametrize("cfg", CONVS)
def test_conv_fwd_bwd(dev, cfg, mode, monkeypatch):
    """conv fwd / dgrad / wgrad vs fp64 torch at 1e-5: the fp16x3 kernels (default for the
    conv2-shaped forward -- 3 tap-row groups, 11-12 kernel columns, width stride 1 -- and the
    4 x 2-fragment dgrad), the bf16x6 direct kernels (DS2_CONV_H3=0, and where fp16x3 does not
    apply: width stride 1, <= 24 tap rows, <= 12 kernel columns) and the fp32 LDS-patch /
    implicit-GEMM kernels (DS2_CONV_X6=0, and every shape the bf16x6 kernels do not cover)."""
    _conv_mode(monkeypatch, mode)
    n, ci, h, w, co, kh, kw, sh, sw, ph, pw = cfg
    g = torch.Generator().manual_seed(sum(cfg))
    x = torch.randn(n, ci, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(co, ci, kh, kw, generator=g, dtype=torch.float64) * 0.1
    bias = torch.randn(co, generator=g, dtype=torch.float64)
    x.requires_grad_(True)
    wt.requires_grad_(True)
    y = F.conv2d(x, wt, bias, stride=(sh, sw), padding=(ph, pw))
    ho, wo = y.shape[2], y.shape[3]
    lens = torch.tensor([wo - 3 * i for i in range(n)], dtype=torch.int32)
    yd = ops.conv2d_fwd(x.detach().float().to(dev), wt.detach().float().to(dev),
                        bias.float().to(dev), (sh, sw), (ph, pw), out_lens=lens.to(dev))
    ref = y.detach().clone()
    for i in range(n):
        ref[i, :, :, int(lens[i]):] = 0
    _close(yd, ref, 1e-5, "conv fwd")
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    y.backward(dy)
    dx = ops.conv2d_dgrad(dy.float().to(dev), wt.detach().float().to(dev), x.shape, (sh, sw),
                          (ph, pw))
    dw, db = ops.conv2d_wgrad(dy.float().to(dev), x.detach().float().to(dev), tuple(wt.shape),
                              (sh, sw), (ph, pw), with_bias=True)
    _close(dx, x.grad, 1e-5, "conv dgrad")
    _close(dw, wt.grad, 1e-5, "conv wgrad")
    _close(db, dy.sum((0, 2, 3)), 1e-5, "conv dbias")


def test_conv_x6_is_fp32_accurate(dev, monkeypatch):
    """On the model's conv2 (32 -> 32 channels, 21 x 11 taps, stride (2, 1)) the fp16x3 and
    bf16x6 kernels' error against fp64 is of the fp32 kernels' order (fwd, dgrad and wgrad)."""
    n, ci, h, w, co, kh, kw, sh, sw, ph, pw = 2, 32, 81, 300, 32, 21, 11, 2, 1, 10, 5
    g = torch.Generator().manual_seed(11)
    x = torch.randn(n, ci, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(co, ci, kh, kw, generator=g, dtype=torch.float64) * 0.1
    y = F.conv2d(x, wt, None, stride=(sh, sw), padding=(ph, pw))
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    dxr = torch.nn.grad.conv2d_input(x.shape, wt, dy, stride=(sh, sw), padding=(ph, pw))
    dwr = torch.nn.grad.conv2d_weight(x, wt.shape, dy, stride=(sh, sw), padding=(ph, pw))
    errs = {}
    for mode in ("h3", "x6", "fp32"):
        _conv_mode(monkeypatch, mode)
        yd = ops.conv2d_fwd(x.float().to(dev), wt.float().to(dev), None, (sh, sw), (ph, pw))
        dx = ops.conv2d_dgrad(dy.float().to(dev), wt.float().to(dev), x.shape, (sh, sw), (ph, pw))
        dw, _ = ops.conv2d_wgrad(dy.float().to(dev), x.float().to(dev), tuple(wt.shape), (sh, sw),
                                 (ph, pw), with_bias=False)
        errs[mode] = tuple((a.double().cpu() - r).abs().max().item() / r.abs().max().item()
                           for a, r in ((yd, y), (dx, dxr), (dw, dwr)))
    for mode in ("h3", "x6"):
        assert all(e1 <= 2.5 * e0 for e1, e0 in zip(errs[mode], errs["fp32"])), errs
        assert max(errs[mode]) < 5e-6, errs


@pytest.mark.parametrize("h,w,n,lens", [(81, 300, 2, None), (81, 501, 3, (501, 377, 120)),
                                        (17, 90, 2, None), (9, 40, 1, None), (31, 260, 2, (200, 260))])
def test_conv2_two_row_forward(dev, h, w, n, lens, monkeypatch):
    """conv_h3_fwd2r_kernel (conv2's fp16x3 forward, output rows r and r + 4 per workgroup from
    one 32-row patch, sign flip per input channel) against the one-row conv_x6_kernel
    (DS2_CONV_2R=0) and fp64: the same fp32-level error (ragged output rows 41 / 9 / 5 / 16,
    partial column blocks, bias, MaskConv lengths), and no systematic drift -- the mean of the
    signed error stays a small fraction of the mean absolute error, as the sign split keeps
    it for the one-row kernel ("MFMA rounding")."""
    ci, co, kh, kw, sh, sw, ph, pw = 32, 32, 21, 11, 2, 1, 10, 5
    g = torch.Generator().manual_seed(h * 1000 + w)
    x = torch.randn(n, ci, h, w, generator=g, dtype=torch.float64).abs() * 3   # conv1 block: >= 0
    wt = torch.randn(co, ci, kh, kw, generator=g, dtype=torch.float64) * 0.05
    b = torch.randn(co, generator=g, dtype=torch.float64)
    ref = F.conv2d(x, wt, b, stride=(sh, sw), padding=(ph, pw))
    ld = None
    if lens is not None:
        ld = torch.tensor(lens, dtype=torch.int32, device=dev)
        for i, L in enumerate(lens):
            ref[i, :, :, L:] = 0.0
    outs = {}
    for two in ("1", "0"):
        monkeypatch.setenv("DS2_CONV_2R", two)
        outs[two] = ops.conv2d_fwd(x.float().to(dev), wt.float().to(dev), b.float().to(dev),
                                   (sh, sw), (ph, pw), out_lens=ld).double().cpu()
    scale = ref.abs().max().item()
    e2 = (outs["1"] - ref).abs().max().item() / scale
    e1 = (outs["0"] - ref).abs().max().item() / scale
    assert e2 < 2e-6 and e2 <= 2.5 * e1 + 1e-7, (e2, e1)
    err = (outs["1"] - ref)[ref != 0]
    drift = (err.mean() / err.abs().mean()).item()
    assert abs(drift) < 0.1, drift


@pytest.mark.parametrize("h,w,n", [(81, 300, 2), (81, 501, 1), (17, 90, 2), (9, 40, 1), (31, 260, 2),
                                   (2, 30, 1)])
def test_conv2_two_row_dgrad(dev, h, w, n, monkeypatch):
    """conv_h3_dgrad2r_kernel (conv2's fp16x3 dgrad, dx rows t and t + 4 of a stride class per
    workgroup from one 16-row dy patch, the big chain restarted per output channel) against the
    one-row conv_x6q_dgrad_kernel (DS2_CONV_2R=0) and fp64: fp32-level error on ragged class row
    counts (41 + 40, 9 + 8, 16 + 15, 5 + 4, 1 + 1 rows), and no systematic drift."""
    ci, co, kh, kw, sh, sw, ph, pw = 32, 32, 21, 11, 2, 1, 10, 5
    g = torch.Generator().manual_seed(h * 1000 + w + 7)
    ho, wo = (h + 2 * ph - kh) // sh + 1, (w + 2 * pw - kw) // sw + 1
    wt = torch.randn(co, ci, kh, kw, generator=g, dtype=torch.float64) * 0.05
    dy = torch.randn(n, co, ho, wo, generator=g, dtype=torch.float64)
    ref = torch.nn.grad.conv2d_input((n, ci, h, w), wt, dy, stride=(sh, sw), padding=(ph, pw))
    outs = {}
    for two in ("1", "0"):
        monkeypatch.setenv("DS2_CONV_2R", two)
        outs[two] = ops.conv2d_dgrad(dy.float().to(dev), wt.float().to(dev), (n, ci, h, w), (sh, sw),
                                     (ph, pw)).double().cpu()
    scale = ref.abs().max().item()
    e2 = (outs["1"] - ref).abs().max().item() / scale
    e1 = (outs["0"] - ref).abs().max().item() / scale
    assert e2 < 2e-6 and e2 <= 2.5 * e1 + 1e-7, (e2, e1)
    err = (outs["1"] - ref)[ref != 0]
    drift = (err.mean() / err.abs().mean()).item()
    assert abs(drift) < 0.1, drift


def test_conv_h3_scales_over_twelve_decades(dev, monkeypatch):
    """fp16x3 conv2 forward / dgrad with samples and output channels spread over 10^+-6, and
    the weight gradient with input and output channels spread likewise: the per-sample input
    scale, per-row weight scale and per-channel wgrad scales keep every output at the fp32
    error bound's form, max |y - y64| / (|w| * |x|) (the same convolution of absolute values),
    within 2.5x of bf16x6's and below 2e-6."""
    n, ci, h, w, co, kh, kw, sh, sw, ph, pw = 4, 32, 81, 90, 32, 21, 11, 2, 1, 10, 5
    g = torch.Generator().manual_seed(23)
    sx = torch.pow(10.0, torch.linspace(-6, 6, n, dtype=torch.float64))
    sw_ = torch.pow(10.0, torch.empty(co, dtype=torch.float64).uniform_(-6, 6, generator=g))
    x = torch.randn(n, ci, h, w, generator=g, dtype=torch.float64) * sx[:, None, None, None]
    wt = torch.randn(co, ci, kh, kw, generator=g, dtype=torch.float64) * 0.1 * sw_[:, None, None, None]
    y = F.conv2d(x, wt, None, stride=(sh, sw), padding=(ph, pw))
    yb = F.conv2d(x.abs(), wt.abs(), None, stride=(sh, sw), padding=(ph, pw))
    # dgrad: dy samples spread the same way, the weight rows of the dgrad GEMM are ci
    swi = torch.pow(10.0, torch.empty(ci, dtype=torch.float64).uniform_(-6, 6, generator=g))
    wt2 = torch.randn(co, ci, kh, kw, generator=g, dtype=torch.float64) * 0.1 * swi[None, :, None, None]
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64) * sx[:, None, None, None]
    dxr = torch.nn.grad.conv2d_input(x.shape, wt2, dy, stride=(sh, sw), padding=(ph, pw))
    dxb = torch.nn.grad.conv2d_input(x.shape, wt2.abs(), dy.abs(), stride=(sh, sw), padding=(ph, pw))
    # wgrad: x channels (ci) and dy channels (co) spread over 10^+-6 -- the fp16x3 weight
    # gradient scales each by its own channel maximum over the batch
    xw = torch.randn(n, ci, h, w, generator=g, dtype=torch.float64) * swi[None, :, None, None]
    dyw = torch.randn(y.shape, generator=g, dtype=torch.float64) * sw_[None, :, None, None]
    dwr = torch.nn.grad.conv2d_weight(xw, wt.shape, dyw, stride=(sh, sw), padding=(ph, pw))
    dwb = torch.nn.grad.conv2d_weight(xw.abs(), wt.shape, dyw.abs(), stride=(sh, sw), padding=(ph, pw))
    errs = {}
    for mode in ("h3", "x6"):
        _conv_mode(monkeypatch, mode)
        yd = ops.conv2d_fwd(x.float().to(dev), wt.float().to(dev), None, (sh, sw), (ph, pw))
        dx = ops.conv2d_dgrad(dy.float().to(dev), wt2.float().to(dev), x.shape, (sh, sw), (ph, pw))
        dwd, _ = ops.conv2d_wgrad(dyw.float().to(dev), xw.float().to(dev), tuple(wt.shape), (sh, sw),
                                  (ph, pw), with_bias=False)
        errs[mode] = tuple(((a.double().cpu() - r).abs() / b.clamp_min(1e-300)).max().item()
                           for a, r, b in ((yd, y, yb), (dx, dxr, dxb), (dwd, dwr, dwb)))
    assert all(e3 <= 2.5 * e6 + 1e-7 for e3, e6 in zip(errs["h3"], errs["x6"])), errs
    assert max(errs["h3"]) < 2e-6, errs


@pytest.mark.parametrize("cfg", [(2, 32, 81, 200, 32, 21, 11, 2, 1, 10, 5),
                                 (3, 5, 30, 70, 20, 7, 11, 1, 1, 3, 5),
                                 (4, 32, 81, 70, 32, 21, 11, 2, 1, 10, 5),
                                 (2, 8, 40, 60, 16, 7, 11, 3, 1, 3, 5)])
@pytest.mark.parametrize("w64", ["0", "1"])
def test_conv_x6_wgrad_forms(dev, cfg, w64, monkeypatch):
    """The bf16x6 weight gradients against fp64 torch: the sliding-window form (row strides
    <= 2: sh new x rows per output row into a 6-slot ring; splits that start mid-segment and
    segments of one row, 4 x 70 columns = 3 chunks per row) and the per-row-restaging form
    (row stride 3).  w64 = 1: the fp16x3 sliding window on 64-column stages (DS2_CONV_W64;
    200 columns = 4 chunks with a partial last one, 70 = 2)."""
    monkeypatch.setenv("DS2_CONV_W64", w64)
    n, ci, h, w, co, kh, kw, sh, sw, ph, pw = cfg
    g = torch.Generator().manual_seed(sum(cfg) + 1)
    x = torch.randn(n, ci, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(co, ci, kh, kw, generator=g, dtype=torch.float64) * 0.1
    y = F.conv2d(x, wt, None, stride=(sh, sw), padding=(ph, pw))
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    dwr = torch.nn.grad.conv2d_weight(x, wt.shape, dy, stride=(sh, sw), padding=(ph, pw))
    dw, _ = ops.conv2d_wgrad(dy.float().to(dev), x.float().to(dev), tuple(wt.shape), (sh, sw),
                             (ph, pw), with_bias=False)
    _close(dw, dwr, 1e-5, "conv wgrad")


# ---------------------------------------------------------------------------- BN
def test_seq_bn_fwd_bwd(dev):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(777, 96, generator=g, dtype=torch.float64) * 3 + 1
    gamma = torch.rand(96, generator=g, dtype=torch.float64) + 0.5
    beta = torch.randn(96, generator=g, dtype=torch.float64)
    rm, rv = torch.zeros(96), torch.ones(96)
    rm_d, rv_d = rm.clone().to(dev), rv.clone().to(dev)
    xr = x.clone().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    y = F.batch_norm(xr, rm.double(), rv.double(), gr, br, training=True, momentum=0.1, eps=1e-5)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    y.backward(dy)
    xd = x.float().to(dev).requires_grad_(True)
    gd = gamma.float().to(dev).requires_grad_(True)
    bd = beta.float().to(dev).requires_grad_(True)
    yd = ops.SeqBatchNormFn.apply(xd, gd, bd, rm_d, rv_d, True, 0.1, 1e-5)
    yd.backward(dy.float().to(dev))
    _close(yd, y, 1e-5, "bn y")
    _close(xd.grad, xr.grad, 1e-4, "bn dx")
    _close(gd.grad, gr.grad, 1e-5, "bn dgamma")
    _close(bd.grad, br.grad, 1e-5, "bn dbeta")
    _close(rm_d, 0.1 * x.mean(0), 1e-5, "running_mean")
    _close(rv_d, 0.9 + 0.1 * x.var(0, unbiased=True), 1e-5, "running_var")


@pytest.mark.parametrize("rows,c", [(32032, 800), (777, 96), (5, 1600), (130, 260), (64, 4)])
def test_bn_apply_amax(dev, rows, c):
    """ds2_bn_apply_amax: y bit-identical to ds2_bn_apply, and its row / column maxima equal to
    |y|'s (the fp16x3 scales the next input projection and dW_ih take from it), for every
    columns-per-lane instantiation and ragged row counts."""
    g = torch.Generator().manual_seed(rows + c)
    x = (torch.randn(rows, c, generator=g) * 3 + 1).to(dev)
    mean, invstd = (torch.randn(c, generator=g).to(dev), (torch.rand(c, generator=g) + .5).to(dev))
    gamma, beta = (torch.randn(c, generator=g).to(dev), torch.randn(c, generator=g).to(dev))
    y0 = ops.bn_apply(x, rows, c, 1, mean, invstd, gamma, beta)
    y1 = ops.bn_apply_amax(x, rows, c, mean, invstd, gamma, beta)
    assert torch.equal(y0, y1)
    rmax, cmax = ops._take_amax(y1, rows, c)
    assert rmax is not None and all(v is None for v in ops._take_amax(y1, rows, c))
    ay = y1.abs()
    assert torch.equal(rmax, ay.amax(1).contiguous().view(torch.int32))
    assert torch.equal(cmax, ay.amax(0).contiguous().view(torch.int32))
    # an in-place change of y invalidates the maxima
    y2 = ops.bn_apply_amax(x, rows, c, mean, invstd, gamma, beta)
    y2.mul_(2)
    assert all(v is None for v in ops._take_amax(y2, rows, c))


@pytest.mark.parametrize("layout", [0, 1])
def test_conv_block_fwd_bwd(dev, layout):
    """ConvBlockFn vs conv2d -> mask -> BN -> mask -> hardtanh -> mask (model.py:63-79)."""
    g = torch.Generator().manual_seed(11 + layout)
    n, ci, h, w = 3, 4, 21, 30
    co, kh, kw, sh, sw, ph, pw = 8, 5, 3, 2, 1, 2, 1
    x = torch.randn(n, ci, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(co, ci, kh, kw, generator=g, dtype=torch.float64) * 0.3
    b = torch.randn(co, generator=g, dtype=torch.float64)
    gamma = torch.rand(co, generator=g, dtype=torch.float64) * 4 + 2
    beta = torch.randn(co, generator=g, dtype=torch.float64) * 3 + 4
    lens = torch.tensor([w, w - 7, w - 13], dtype=torch.int32)
    params = [t.clone().requires_grad_(True) for t in (x, wt, b, gamma, beta)]
    xr, wr, brr, gr, ber = params
    rm, rv = torch.zeros(co, dtype=torch.float64), torch.ones(co, dtype=torch.float64)

    def mask(t):
        m = torch.arange(t.shape[-1])[None, :] >= lens[:, None].long()
        return t.masked_fill(m[:, None, None, :], 0)
    z = mask(F.conv2d(xr, wr, brr, stride=(sh, sw), padding=(ph, pw)))
    z = mask(F.batch_norm(z, rm, rv, gr, ber, training=True, momentum=0.1, eps=1e-5))
    y = mask(F.hardtanh(z, 0, 20))
    nn_, c_, d_, t_ = y.shape
    yref = y if layout == 0 else y.reshape(nn_, c_ * d_, t_).permute(2, 0, 1)
    dy = torch.randn(yref.shape, generator=g, dtype=torch.float64)
    yref.backward(dy)
    dparams = [p.detach().float().to(dev).requires_grad_(True) for p in params]
    xd, wd, bd, gd, bed = dparams
    rm_d, rv_d = torch.zeros(co, device=dev), torch.ones(co, device=dev)
    yd = ops.ConvBlockFn.apply(xd, lens.to(dev), wd, bd, gd, bed, rm_d, rv_d, True, 0.1, 1e-5,
                               (sh, sw), (ph, pw), 0.0, 20.0, layout)
    yd.backward(dy.float().to(dev))
    _close(yd, yref, 1e-5, "block y")
    for name, pd, pr in zip(["dx", "dw", "dbias", "dgamma", "dbeta"], dparams, params):
        _close(pd.grad, pr.grad, 2e-4, name)


@pytest.mark.parametrize("mode", ["h3", "x6", "fp32"])
def test_conv_block_model_conv2_ragged(dev, mode, monkeypatch):
    """ConvBlockFn at the model's conv2 (32 -> 32 channels, 21 x 11 taps, stride (2, 1), the
    input a Hardtanh(0, 20) output) with ragged lengths -- the kernels the bs32 benchmark uses
    (fp16x3 forward / dgrad, sliding-window wgrad), with the time mask of model.py:69-78 --
    vs fp64: output 1e-5, gradients 2e-4 (relative to max), in each conv mode."""
    _conv_mode(monkeypatch, mode)
    g = torch.Generator().manual_seed(23)
    n, ci, h, w = 3, 32, 41, 150
    co, kh, kw, sh, sw, ph, pw = 32, 21, 11, 2, 1, 10, 5
    lens = torch.tensor([w, w - 31, 62], dtype=torch.int32)
    x = (torch.rand(n, ci, h, w, generator=g, dtype=torch.float64) * 24 - 2).clamp(0, 20)
    for i in range(n):
        x[i, :, :, int(lens[i]):] = 0
    wt = torch.randn(co, ci, kh, kw, generator=g, dtype=torch.float64) * (ci * kh * kw) ** -0.5
    b = torch.randn(co, generator=g, dtype=torch.float64) * 0.1
    gamma = torch.rand(co, generator=g, dtype=torch.float64) + 0.5
    beta = torch.randn(co, generator=g, dtype=torch.float64) * 0.2
    params = [t.clone().requires_grad_(True) for t in (x, wt, b, gamma, beta)]
    xr, wr, brr, gr, ber = params
    rm, rv = torch.zeros(co, dtype=torch.float64), torch.ones(co, dtype=torch.float64)

    def mask(t):
        m = torch.arange(t.shape[-1])[None, :] >= lens[:, None].long()
        return t.masked_fill(m[:, None, None, :], 0)
    z = mask(F.conv2d(xr, wr, brr, stride=(sh, sw), padding=(ph, pw)))
    z = mask(F.batch_norm(z, rm, rv, gr, ber, training=True, momentum=0.1, eps=1e-5))
    y = mask(F.hardtanh(z, 0, 20))
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    y.backward(dy)
    dparams = [p.detach().float().to(dev).requires_grad_(True) for p in params]
    xd, wd, bd, gd, bed = dparams
    rm_d, rv_d = torch.zeros(co, device=dev), torch.ones(co, device=dev)
    yd = ops.ConvBlockFn.apply(xd, lens.to(dev), wd, bd, gd, bed, rm_d, rv_d, True, 0.1, 1e-5,
                               (sh, sw), (ph, pw), 0.0, 20.0, 0)
    yd.backward(dy.float().to(dev))
    _close(yd, y, 1e-5, "block y")
    for name, pd, pr in zip(["dx", "dw", "dbias", "dgamma", "dbeta"], dparams, params):
        _close(pd.grad, pr.grad, 2e-4, name)


# ---------------------------------------------------------------------------- GRU
@pytest.mark.parametrize("n,t,inp,h,bidir", [(5, 23, 40, 24, True), (19, 9, 33, 400, True),
                                             (3, 17, 20, 16, False), (20, 30, 64, 800, True),
                                             (6, 12, 32, 1024, True)])
def test_gru_layer(dev, n, t, inp, h, bidir):
    g = torch.Generator().manual_seed(n * 100 + h)
    gru = torch.nn.GRU(inp, h, bidirectional=bidir).double()
    # +-0.3 for the small layers; the PyTorch default range 1/sqrt(h) for h = 800, where
    # +-0.3 makes the recurrence chaotic enough that fp32 and fp64 trajectories separate
    a = 0.3 if h <= 400 else h ** -0.5
    with torch.no_grad():
        for p in gru.parameters():
            p.copy_((torch.rand(p.shape, generator=g, dtype=torch.float64) * 2 - 1) * a)
    lens = torch.tensor(sorted([t] + [max(1, t - 3 * i - 1) for i in range(n - 1)], reverse=True),
                        dtype=torch.int32)
    x = torch.randn(t, n, inp, generator=g, dtype=torch.float64)
    for i in range(n):
        x[int(lens[i]):, i] = 0
    xr = x.clone().requires_grad_(True)
    packed = torch.nn.utils.rnn.pack_padded_sequence(xr, lens.numpy())
    out, _ = gru(packed)
    out, _ = torch.nn.utils.rnn.pad_packed_sequence(out, total_length=t)
    nd = 2 if bidir else 1
    summed = out.view(t, n, nd, h).sum(2) if bidir else out
    dy = torch.randn(summed.shape, generator=g, dtype=torch.float64)
    summed.backward(dy)
    weights = [p.detach().float().to(dev).requires_grad_(True) for p in gru.parameters()]
    xd = x.float().to(dev).requires_grad_(True)
    yd = ops.GRULayerFn.apply(xd, lens.to(dev), True, h, *weights)
    yd.backward(dy.float().to(dev))
    _close(yd, summed, 1e-5, "gru y")
    _close(xd.grad, xr.grad, 1e-4, "gru dx")
    for (name, p), wd in zip(gru.named_parameters(), weights):
        _close(wd.grad, p.grad, 1e-4, "gru " + name)


@pytest.mark.parametrize("h", [24, 400])
def test_gru_persistent_equals_per_step(dev, h, monkeypatch):
    """The persistent (one launch per layer) and per-step-launch recurrences agree (their
    K split over waves may differ, so the fp32 summation order can differ)."""
    n, t, inp = 21, 37, 48
    g = torch.Generator().manual_seed(h)
    weights = [torch.rand(s, generator=g) * 0.4 - 0.2 for s in
               [(3 * h, inp), (3 * h, h), (3 * h,), (3 * h,)] * 2]
    lens = torch.tensor(sorted([t - (i % 7) * 3 for i in range(n)], reverse=True), dtype=torch.int32)
    x = torch.randn(t, n, inp, generator=g)
    dy = torch.randn(t, n, h, generator=g)
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("DS2_RNN_PERSISTENT", flag)
        ws = [w.to(dev).requires_grad_(True) for w in weights]
        xd = x.to(dev).requires_grad_(True)
        y = ops.GRULayerFn.apply(xd, lens.to(dev), True, h, *ws)
        y.backward(dy.to(dev))
        torch.cuda.synchronize()
        outs.append([y.detach().cpu(), xd.grad.cpu()] + [w.grad.cpu() for w in ws])
    for a, b in zip(*outs):
        _close(a, b, 1e-5, "persistent vs per-step")


@pytest.mark.parametrize("n,h,bidir", [(32, 800, True), (20, 64, True), (7, 48, False),
                                       (17, 784, True), (16, 1024, True)])
def test_gru_bf16x6_matches_fp32_mfma(dev, n, h, bidir, monkeypatch):
    """gru_split.hip (W_hh contraction as six bf16 products of three-term splits, fp32
    accumulation; sentinel-ring forward, pre-split flag backward) against the fp32-MFMA
    direct-operand kernels (DS2_GRU_X6=0): equal within fp32 rounding (different summation
    order; odd UB = 49 included: the last 32-k pair is half empty)."""
    nd = 2 if bidir else 1
    env = [{"DS2_GRU_X6": "0"},
           {"DS2_GRU_X6": "1", "DS2_GRU_H3": "0", "DS2_GRU_H3_BWD": "0"},
           {"DS2_GRU_X6": "1", "DS2_GRU_H3": "1", "DS2_GRU_H3_BWD": "1"}]
    f32, x6, h3 = _gru_run(dev, n, 41, 40, h, nd, h + 7 * n, env, monkeypatch)
    for a, b, c in zip(f32, x6, h3):
        assert torch.isfinite(b).all() and torch.isfinite(c).all()
        _close(b, a, 2e-5, "bf16x6 vs fp32 MFMA")
        _close(c, a, 2e-5, "fp16x3 recurrences vs fp32 MFMA")


def _gru_run(dev, n, t, inp, h, nd, seed, env, monkeypatch, amp=None):
    g = torch.Generator().manual_seed(seed)
    a = amp if amp is not None else (0.2 if h <= 64 else h ** -0.5)
    weights = [torch.rand(s, generator=g) * 2 * a - a for s in
               [(3 * h, inp), (3 * h, h), (3 * h,), (3 * h,)] * nd]
    lens = torch.tensor(sorted([t - (i % 6) * 5 for i in range(n)], reverse=True),
                        dtype=torch.int32)
    x = torch.randn(t, n, inp, generator=g)
    dy = torch.randn(t, n, h, generator=g)
    outs = []
    for e in env:
        for k, v in e.items():
            monkeypatch.setenv(k, v)
        ws = [w.to(dev).requires_grad_(True) for w in weights]
        xd = x.to(dev).requires_grad_(True)
        y = ops.GRULayerFn.apply(xd, lens.to(dev), True, h, *ws)
        y.backward(dy.to(dev))
        torch.cuda.synchronize()
        ops.check_rnn_status(dev)
        outs.append([y.detach().cpu(), xd.grad.cpu()] + [w.grad.cpu() for w in ws])
    return outs


@pytest.mark.parametrize("kern", ["h3", "x6"])
@pytest.mark.parametrize("n,h,bidir", [(32, 800, True), (7, 48, False), (17, 784, True),
                                       (33, 256, True), (16, 1024, True), (64, 256, False)])
def test_gru_xcd_groups_bit_identical(dev, n, h, bidir, kern, monkeypatch):
    """The same-XCD hand-off groups (default where the groups tile the 8 XCDs: 32 x 800 and
    16 x 1024 bidirectional, 64 x 256 unidirectional) read the same bytes from plainly stored
    copies, placed by the XCC id each producer publishes: outputs and gradients bit-identical
    to the interleaved layout (DS2_GRU_XCD=0), ragged lengths; for the fp16x3 recurrences
    (default) and the bf16x6 ones."""
    nd = 2 if bidir else 1
    f = "1" if kern == "h3" else "0"
    monkeypatch.setenv("DS2_GRU_XL", "0")    # the 16-unit kernels' groups
    monkeypatch.setenv("DS2_GRU_H3", f)
    monkeypatch.setenv("DS2_GRU_H3_BWD", f)
    env = [{"DS2_GRU_XCD": "1"}, {"DS2_GRU_XCD": "0"}]
    xg, il = _gru_run(dev, n, 37, 40, h, nd, h + 13 * n, env, monkeypatch)
    for a, b in zip(xg, il):
        assert torch.isfinite(a).all()
        assert torch.equal(a, b)


@pytest.mark.parametrize("n,h,bidir", [(32, 800, True), (13, 800, True), (20, 64, True),
                                       (64, 256, False), (8, 32, False), (3, 96, True)])
def test_gru_xl_matches_16unit_kernels(dev, n, h, bidir, monkeypatch):
    """The XCD-local recurrences (gru_xl.hip: 32 units x 8 samples per workgroup, a group of
    H / 32 workgroups in one XCD, stacked (hi; lo) fp16 fragments; the default where they fit)
    against the 16-unit fp16x3 kernels (DS2_GRU_XL=0) and the fp32-MFMA ones (DS2_GRU_X6=0):
    equal within fp32 rounding, ragged lengths, partial batch tiles (13, 3 samples), one and
    two directions, 1 to 25 producers per group; a second XL run is bit-identical (the sums
    run in a fixed producer order whatever the arrival order)."""
    nd = 2 if bidir else 1
    env = [{"DS2_GRU_XL": "1"}, {"DS2_GRU_XL": "1"}, {"DS2_GRU_XL": "0"},
           {"DS2_GRU_XL": "1", "DS2_GRU_X6": "0"}]
    xl, xl2, h3, f32 = _gru_run(dev, n, 41, 40, h, nd, h + 11 * n, env, monkeypatch)
    for a, b, c, d in zip(xl, xl2, h3, f32):
        assert torch.isfinite(a).all()
        assert torch.equal(a, b)
        _close(a, c, 2e-5, "XCD-local vs 16-unit fp16x3")
        _close(a, d, 2e-5, "XCD-local vs fp32 MFMA")


@pytest.mark.parametrize("n,h,bidir", [(32, 800, True), (64, 256, False)])
def test_gru_xl_local_equals_global(dev, n, h, bidir, monkeypatch):
    """A group whose workgroups share one XCD publishes with plain stores (kept in that XCD's
    L2); DS2_GRU_XL=2 makes every group publish write-through (sc1), the placement-independent
    form it falls back to when its members' XCC ids differ: same bytes, bit-identical."""
    nd = 2 if bidir else 1
    env = [{"DS2_GRU_XL": "1"}, {"DS2_GRU_XL": "2"}]
    loc, glob = _gru_run(dev, n, 37, 40, h, nd, h + 5 * n, env, monkeypatch)
    for a, b in zip(loc, glob):
        assert torch.isfinite(a).all()
        assert torch.equal(a, b)


@pytest.mark.parametrize("x6", ["1", "0", "x6"])
def test_gru_backward_full_length_vs_torch(dev, x6, monkeypatch):
    """The cfg2 recurrence shape (bs 32, H 800, both directions) over 201 steps with ragged
    lengths: the default recurrences (fp16x3 forward and backward), the bf16x6 ones
    (DS2_GRU_H3=0 DS2_GRU_H3_BWD=0, "x6") and the fp32-MFMA kernels (DS2_GRU_X6=0) against
    torch's nn.GRU in fp64."""
    monkeypatch.setenv("DS2_GRU_X6", "0" if x6 == "0" else "1")
    monkeypatch.setenv("DS2_GRU_H3", "0" if x6 == "x6" else "1")
    monkeypatch.setenv("DS2_GRU_H3_BWD", "0" if x6 == "x6" else "1")
    n, t, inp, h = 32, 201, 64, 800
    g = torch.Generator().manual_seed(3)
    gru = torch.nn.GRU(inp, h, bidirectional=True).double()
    with torch.no_grad():
        for p in gru.parameters():
            p.copy_((torch.rand(p.shape, generator=g, dtype=torch.float64) * 2 - 1) * h ** -0.5)
    lens = torch.tensor(sorted([t - 6 * i for i in range(n)], reverse=True), dtype=torch.int32)
    x = torch.randn(t, n, inp, generator=g, dtype=torch.float64)
    for i in range(n):
        x[int(lens[i]):, i] = 0
    xr = x.clone().requires_grad_(True)
    out, _ = gru(torch.nn.utils.rnn.pack_padded_sequence(xr, lens.numpy()))
    out, _ = torch.nn.utils.rnn.pad_packed_sequence(out, total_length=t)
    summed = out.view(t, n, 2, h).sum(2)
    dy = torch.randn(summed.shape, generator=g, dtype=torch.float64)
    summed.backward(dy)
    weights = [p.detach().float().to(dev).requires_grad_(True) for p in gru.parameters()]
    xd = x.float().to(dev).requires_grad_(True)
    yd = ops.GRULayerFn.apply(xd, lens.to(dev), True, h, *weights)
    yd.backward(dy.float().to(dev))
    ops.check_rnn_status(dev)
    _close(yd, summed, 1e-5, "gru y")
    _close(xd.grad, xr.grad, 1e-4, "gru dx")
    for (name, p), wd in zip(gru.named_parameters(), weights):
        _close(wd.grad, p.grad, 1e-4, "gru " + name)


def test_gru_per_direction_output(dev):
    n, t, inp, h = 4, 11, 8, 16
    g = torch.Generator().manual_seed(5)
    gru = torch.nn.GRU(inp, h, bidirectional=True).double()
    lens = torch.tensor([11, 9, 4, 1], dtype=torch.int32)
    x = torch.randn(t, n, inp, generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    out, _ = gru(torch.nn.utils.rnn.pack_padded_sequence(xr, lens.numpy()))
    out, _ = torch.nn.utils.rnn.pad_packed_sequence(out, total_length=t)
    dy = torch.randn(out.shape, generator=g, dtype=torch.float64)
    out.backward(dy)
    weights = [p.detach().float().to(dev).requires_grad_(True) for p in gru.parameters()]
    xd = x.float().to(dev).requires_grad_(True)
    yd = ops.GRULayerFn.apply(xd, lens.to(dev), False, h, *weights)
    yd.backward(dy.float().to(dev))
    _close(yd, out, 1e-5, "gru y")
    _close(xd.grad, xr.grad, 1e-4, "gru dx")


# ---------------------------------------------------------------------------- tanh RNN
@pytest.mark.parametrize("persistent", ["1", "0"])
@pytest.mark.parametrize("n,t,inp,h,bidir", [(5, 23, 40, 24, True), (19, 9, 33, 100, True),
                                             (3, 17, 20, 16, False), (33, 40, 64, 800, True),
                                             (20, 31, 24, 48, True), (32, 120, 96, 800, False)])
def test_rnn_layer(dev, n, t, inp, h, bidir, persistent, monkeypatch):
    """rnn_type 'rnn' (model.py:15, nn.RNN tanh): the ds2amd layer == pack -> nn.RNN -> pad
    (-> direction sum) in fp64, forward and every gradient; ragged lengths, three batch
    tiles of 16 at n = 33.  Both recurrence paths: the one-gate fp16x3 persistent kernels
    (H % 16 == 0: 16, 48, 800; the others fall back) and the per-step kernels
    (DS2_RNN_PERSISTENT=0)."""
    monkeypatch.setenv("DS2_RNN_PERSISTENT", persistent)
    g = torch.Generator().manual_seed(n * 100 + h + 1)
    rnn = torch.nn.RNN(inp, h, bidirectional=bidir).double()
    a = 0.3 if h <= 100 else h ** -0.5
    with torch.no_grad():
        for p in rnn.parameters():
            p.copy_((torch.rand(p.shape, generator=g, dtype=torch.float64) * 2 - 1) * a)
    lens = torch.tensor(sorted([t] + [max(1, t - 3 * i - 1) for i in range(n - 1)], reverse=True),
                        dtype=torch.int32)
    x = torch.randn(t, n, inp, generator=g, dtype=torch.float64)
    for i in range(n):
        x[int(lens[i]):, i] = 0
    xr = x.clone().requires_grad_(True)
    out, _ = rnn(torch.nn.utils.rnn.pack_padded_sequence(xr, lens.numpy()))
    out, _ = torch.nn.utils.rnn.pad_packed_sequence(out, total_length=t)
    nd = 2 if bidir else 1
    summed = out.view(t, n, nd, h).sum(2) if bidir else out
    dy = torch.randn(summed.shape, generator=g, dtype=torch.float64)
    summed.backward(dy)
    weights = [p.detach().float().to(dev).requires_grad_(True) for p in rnn.parameters()]
    xd = x.float().to(dev).requires_grad_(True)
    yd = ops.RNNLayerFn.apply(xd, lens.to(dev), True, h, *weights)
    yd.backward(dy.float().to(dev))
    _close(yd, summed, 1e-5, "rnn y")
    _close(xd.grad, xr.grad, 1e-4, "rnn dx")
    for (name, p), wd in zip(rnn.named_parameters(), weights):
        _close(wd.grad, p.grad, 1e-4, "rnn " + name)


# ---------------------------------------------------------------------------- LSTM
def _lstm_case(n, t, inp, h, bidir, seed):
    g = torch.Generator().manual_seed(seed)
    lstm = torch.nn.LSTM(inp, h, bidirectional=bidir).double()
    with torch.no_grad():
        for p in lstm.parameters():
            p.copy_(torch.rand(p.shape, generator=g, dtype=torch.float64) * 0.2 - 0.1)
    lens = torch.tensor(sorted([t] + [max(1, t - 2 * i - 1) for i in range(n - 1)], reverse=True),
                        dtype=torch.int32)
    x = torch.randn(t, n, inp, generator=g, dtype=torch.float64)
    for i in range(n):
        x[int(lens[i]):, i] = 0
    return lstm, lens, x, g


@pytest.mark.parametrize("h3", ["1", "0"])
@pytest.mark.parametrize("n,t,inp,h,bidir", [(5, 23, 40, 24, True), (19, 9, 33, 400, True),
                                             (3, 17, 20, 16, False),
                                             (64, 5, 64, 1024, True),     # cfg4 shape: 2 batch chunks
                                             (32, 6, 48, 1024, False),    # persistent, 2 bwd chunks
                                             (40, 150, 32, 1024, True)])  # long: 3 tiles, 2 chunks
def test_lstm_layer(dev, n, t, inp, h, bidir, h3, monkeypatch):
    """ds2amd LSTM layer == pack -> nn.LSTM -> pad (-> direction sum), fwd and bwd: the
    fp16x3 recurrences (default; H % 16 == 0) and the fp32-MFMA ones (DS2_LSTM_H3=0)."""
    monkeypatch.setenv("DS2_LSTM_H3", h3)
    lstm, lens, x, g = _lstm_case(n, t, inp, h, bidir, n * 100 + h)
    xr = x.clone().requires_grad_(True)
    out, _ = lstm(torch.nn.utils.rnn.pack_padded_sequence(xr, lens.numpy()))
    out, _ = torch.nn.utils.rnn.pad_packed_sequence(out, total_length=t)
    nd = 2 if bidir else 1
    summed = out.view(t, n, nd, h).sum(2) if bidir else out
    dy = torch.randn(summed.shape, generator=g, dtype=torch.float64)
    summed.backward(dy)
    weights = [p.detach().float().to(dev).requires_grad_(True) for p in lstm.parameters()]
    xd = x.float().to(dev).requires_grad_(True)
    yd = ops.LSTMLayerFn.apply(xd, lens.to(dev), True, h, *weights)
    yd.backward(dy.float().to(dev))
    _close(yd, summed, 1e-5, "lstm y")
    _close(xd.grad, xr.grad, 1e-4, "lstm dx")
    for (name, p), wd in zip(lstm.named_parameters(), weights):
        _close(wd.grad, p.grad, 1e-4, "lstm " + name)


@pytest.mark.parametrize("h,n", [(24, 21), (800, 21), (1024, 40)])
def test_lstm_persistent_equals_per_step(dev, h, n, monkeypatch):
    """Persistent launches (for h = 1024, n = 40: 3 batch tiles run as a 2-tile chunk and a
    1-tile chunk, bidirectional) equal the one-launch-per-step kernels."""
    t, inp = 19, 40
    lstm, lens, x, g = _lstm_case(n, t, inp, h, True, h)
    weights = [p.detach().float() for p in lstm.parameters()]
    x = x.float()
    dy = torch.randn(t, n, h, generator=g)
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("DS2_RNN_PERSISTENT", flag)
        ws = [w.to(dev).requires_grad_(True) for w in weights]
        xd = x.to(dev).requires_grad_(True)
        y = ops.LSTMLayerFn.apply(xd, lens.to(dev), True, h, *ws)
        y.backward(dy.to(dev))
        torch.cuda.synchronize()
        outs.append([y.detach().cpu(), xd.grad.cpu()] + [w.grad.cpu() for w in ws])
    for a, b in zip(*outs):
        _close(a, b, 1e-5, "lstm persistent vs per-step")


@pytest.mark.parametrize("n,t,h,bidir", [(64, 60, 1024, True), (40, 37, 256, False), (7, 9, 48, True),
                                         (5, 8, 40, True)])
def test_lstm_bwd_half_vs_fp32(dev, n, t, h, bidir):
    """ds2_lstm_bwd_half (cfg4's bf16 mode: the backward recurrence's W_hh^T product on one
    fp16 term per operand, 32-sample workgroups, one launch for batch 64) against ds2_lstm_bwd
    (fp32-accurate) on the same forward cache: the gate gradients within 4e-3 of their max
    (11-bit operands, per-row / per-column power-of-two scales), every step finite, ragged
    lengths; a shape it declines falls back to ds2_lstm_bwd exactly."""
    nd = 2 if bidir else 1
    g = torch.Generator().manual_seed(n + t + h)
    xproj = (torch.randn(t, n, nd, 4 * h, generator=g) * 0.5).to(dev)
    w = [((torch.rand(4 * h, h, generator=g) * 2 - 1) * h ** -0.5).to(dev) for _ in range(nd)]
    b = [(torch.rand(4 * h, generator=g) * 0.2 - 0.1).to(dev) for _ in range(nd)]
    lens = torch.tensor(sorted([max(1, t - (i * 5) % t) for i in range(n)], reverse=True),
                        dtype=torch.int32, device=dev)
    h_all = torch.empty(t, n, nd, h, device=dev)
    c_all = torch.empty(t, n, nd, h, device=dev)
    gates = torch.empty(t, n, nd, 4 * h, device=dev)
    st = ops.rnn_status_word(dev)
    ws = ops._ws(_lib.size("ds2_lstm_fwd_workspace_size", n, h, nd), dev)
    wr = w[1].data_ptr() if bidir else None
    br = b[1].data_ptr() if bidir else None
    _lib.call("ds2_lstm_fwd", t, n, h, nd, xproj.data_ptr(), w[0].data_ptr(), wr, b[0].data_ptr(),
              br, lens.data_ptr(), h_all.data_ptr(), c_all.data_ptr(), gates.data_ptr(),
              st.data_ptr(), ws.data_ptr(), ws.numel(), ops._stream())
    dy = torch.randn(t, n, nd, h, generator=g).to(dev)
    out = {}
    for fn in ("ds2_lstm_bwd", "ds2_lstm_bwd_half"):
        dg = torch.full((t, n, nd, 4 * h), 7.0, device=dev)
        wsb = ops._ws(_lib.size("ds2_lstm_bwd_workspace_size", n, h, nd), dev)
        _lib.call(fn, t, n, h, nd, dy.data_ptr(), nd, w[0].data_ptr(), wr, c_all.data_ptr(),
                  gates.data_ptr(), lens.data_ptr(), dg.data_ptr(), st.data_ptr(), wsb.data_ptr(),
                  wsb.numel(), ops._stream())
        torch.cuda.synchronize()
        out[fn] = dg.cpu()
    ops.check_rnn_status(dev)
    ref, got = out["ds2_lstm_bwd"], out["ds2_lstm_bwd_half"]
    assert torch.isfinite(got).all()
    for i in range(n):   # rows past a sample's length are zero on both sides
        assert (got[int(lens[i]):, i] == 0).all()
    err = (got - ref).abs().max().item() / ref.abs().max().item()
    assert err < 4e-3, err
    if h % 16 != 0:
        assert torch.equal(got, ref)


@pytest.mark.parametrize("n,h,bidir", [(64, 1024, True), (21, 800, True), (16, 256, False),
                                       (7, 48, False)])
def test_lstm_xcd_groups_bit_identical(dev, n, h, bidir, monkeypatch):
    """The persistent LSTM backward's same-XCD group placement (64 x 1024 bidirectional: the
    cfg4 shape, two 2-tile chunks; 21 x 800 ragged rows; 16 x 256 unidirectional; 7 x 48 does
    not tile the XCDs and keeps the interleaved layout): outputs and gradients bit-identical to
    DS2_GRU_XCD=0."""
    t, inp = 29, 40
    lstm, lens, x, g = _lstm_case(n, t, inp, h, bidir, h + n)
    weights = [p.detach().float() for p in lstm.parameters()]
    x = x.float()
    dy = torch.randn(t, n, h, generator=g)
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("DS2_GRU_XCD", flag)
        ws = [w.to(dev).requires_grad_(True) for w in weights]
        xd = x.to(dev).requires_grad_(True)
        y = ops.LSTMLayerFn.apply(xd, lens.to(dev), True, h, *ws)
        y.backward(dy.to(dev))
        torch.cuda.synchronize()
        ops.check_rnn_status(dev)
        outs.append([y.detach().cpu(), xd.grad.cpu()] + [w.grad.cpu() for w in ws])
    for a, b in zip(*outs):
        assert torch.isfinite(a).all()
        assert torch.equal(a, b)


# ---------------------------------------------------------------------------- Lookahead
@pytest.mark.parametrize("t,n,h,context", [(37, 3, 20, 20), (7, 2, 33, 20), (50, 5, 130, 3),
                                           (1, 1, 1, 1)])
@pytest.mark.parametrize("fused", [False, True])
def test_lookahead(dev, t, n, h, context, fused):
    """ds2_lookahead_fwd/bwd vs the reference formulation (oracle.lookahead, model.py:158-172),
    optionally fused with Hardtanh(0, 20) (model.py:329-333)."""
    g = torch.Generator().manual_seed(t * 31 + h)
    x = (torch.randn(t, n, h, generator=g, dtype=torch.float64) * 8 + 4)
    w = torch.rand(h, context + 1, generator=g, dtype=torch.float64) - 0.3
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    yr = orc.lookahead(xr, wr)
    if fused:
        yr = torch.nn.functional.hardtanh(yr, 0, 20)
    dy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    yr.backward(dy)
    xd = x.float().to(dev).requires_grad_(True)
    wd = w.float().to(dev).requires_grad_(True)
    yd = ops.LookaheadFn.apply(xd, wd, (0.0, 20.0) if fused else None)
    yd.backward(dy.float().to(dev))
    _close(yd, yr, 1e-5, "lookahead y")
    if fused:
        # the clamp's gradient mask must agree exactly where the output is not at a bound
        inside = (yr.detach() > 0) & (yr.detach() < 20)
        assert torch.equal((yd.detach().cpu() > 0) & (yd.detach().cpu() < 20), inside)
    _close(xd.grad, xr.grad, 1e-5, "lookahead dx")
    _close(wd.grad, wr.grad, 1e-5, "lookahead dw")


# ---------------------------------------------------------------------------- CTC
@pytest.mark.parametrize("t,act,lab", [
    (60, [60, 55, 40, 12, 30, 5], [20, 1, 0, 5, 14, 2]),
    # several 32-step log-prob chunks of the scan; lengths on and next to chunk edges
    (160, [160, 128, 97, 64, 33, 32], [70, 40, 30, 20, 10, 31])])
def test_ctc_vs_torch(dev, t, act, lab):
    g = torch.Generator().manual_seed(9)
    n, c = 6, 30
    acts = torch.randn(t, n, c, generator=g) * 3
    act_lens = torch.tensor(act, dtype=torch.int32)
    label_lens = torch.tensor(lab, dtype=torch.int32)
    labels = torch.randint(1, c, (int(label_lens.sum()),), generator=g, dtype=torch.int32)
    labels[3:6] = 7                       # repeats inside sample 0
    loss_ref, grad_ref = orc.ctc_loss(acts.double(), labels, act_lens, label_lens)
    costs_ref = orc.ctc_costs(acts, labels, act_lens, label_lens)
    costs, grads = ops.ctc_loss_raw(acts.to(dev), labels.to(dev), act_lens.to(dev),
                                    label_lens.to(dev), int(label_lens.max()))
    _close(costs, costs_ref, 1e-5, "ctc costs")
    # alpha/beta live in fp32 log space (warp-ctc's arithmetic class): |alpha| ~ nll ~ 1e2
    # (~5e2 for the 160-step case) carries ~1e-5 (~5e-5) absolute rounding into
    # exp(alpha + beta + nll); grads are O(1).
    _close(grads, grad_ref, 2e-4 if t <= 64 else 5e-4, "ctc grads")


def test_ctc_rescaled_scan_at_the_benchmark_length(dev):
    """The bench's CTC shape (T' = 501, 150-label targets, 29 classes; random logits, so
    |log p| ~ 1.5e3): the scans store each row minus the previous row's maximum and sum the
    shifts in fp64, so exp(alpha + beta + nll - lp) is formed from O(1) fp32 values.  Unscaled
    log-space rows of magnitude ~|log p| put a ~1e-4 relative error on every gradient term (the
    norm shift the train-step tests saw); here the gradients are within 1e-4 (measured 4.8e-5)
    and the costs within 1e-6 of the fp64 oracle, ragged lengths (one sample at T' = 150, one
    label set of length 1) included.  The unscaled scans measured 6.8e-4 on this case, torch's
    CPU ctc_loss in fp32 7.1e-4 (profiles/r9k_ctc_rescale.txt)."""
    g = torch.Generator().manual_seed(21)
    t, n, c = 501, 4, 29
    acts = torch.randn(t, n, c, generator=g) * 2
    act_lens = torch.tensor([501, 438, 254, 150], dtype=torch.int32)
    label_lens = torch.tensor([150, 120, 1, 60], dtype=torch.int32)
    labels = torch.randint(1, c, (int(label_lens.sum()),), generator=g, dtype=torch.int32)
    loss_ref, grad_ref = orc.ctc_loss(acts.double(), labels, act_lens, label_lens)
    costs_ref = orc.ctc_costs(acts.double(), labels, act_lens, label_lens)
    costs, grads = ops.ctc_loss_raw(acts.to(dev), labels.to(dev), act_lens.to(dev),
                                    label_lens.to(dev), int(label_lens.max()))
    cerr = ((costs.double().cpu() - costs_ref.double()).abs() / costs_ref.double().abs()).max().item()
    gerr = ((grads.double().cpu() - grad_ref.double()).abs().max()
            / grad_ref.double().abs().max()).item()
    _, grad32 = orc.ctc_loss(acts, labels, act_lens, label_lens)      # torch's CPU CTC in fp32
    g32err = ((grad32.double() - grad_ref.double()).abs().max()
              / grad_ref.double().abs().max()).item()
    print(f"ctc at T'=501: costs rel {cerr:.2e}, grads max-abs/max-abs {gerr:.2e} "
          f"(torch fp32 CTC: {g32err:.2e})")
    assert cerr <= 1e-6
    assert gerr <= 1e-4


def test_ctc_infeasible_and_module(dev):
    from ds2amd.ctc import CTCLoss
    acts = torch.randn(4, 2, 5)
    labels = torch.tensor([1, 2, 3, 1, 1], dtype=torch.int32)   # sample1 '1 1' needs 3 frames
    act_lens = torch.tensor([4, 2], dtype=torch.int32)
    label_lens = torch.tensor([3, 2], dtype=torch.int32)
    costs, grads = ops.ctc_loss_raw(acts.to(dev), labels.to(dev), act_lens.to(dev),
                                    label_lens.to(dev), 3)
    assert torch.isinf(costs[1]).item() and torch.isfinite(costs[0]).item()
    assert grads[:, 1].abs().sum().item() == 0
    crit = CTCLoss(zero_infinity=True)
    a = acts.to(dev).requires_grad_(True)
    loss = crit(a, labels, act_lens, label_lens)
    loss.backward()
    ref0 = orc.ctc_costs(acts[:, :1], labels[:3], act_lens[:1], label_lens[:1])
    _close(loss, ref0, 1e-5, "zero_infinity sum")
    assert torch.isfinite(a.grad).all().item()


# ---------------------------------------------------------------------------- softmax / greedy
def test_softmax_tnc(dev):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(17, 5, 30, generator=g, dtype=torch.float64) * 4
    xd = x.float().to(dev).requires_grad_(True)
    p = ops.SoftmaxTNCFn.apply(xd)
    ref = F.softmax(x.transpose(0, 1), -1)
    _close(p, ref, 1e-6, "softmax")
    dp = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    p.backward(dp.float().to(dev))
    xr = x.clone().requires_grad_(True)
    F.softmax(xr.transpose(0, 1), -1).backward(dp)
    _close(xd.grad, xr.grad, 1e-5, "softmax bwd")


def test_greedy_decode_bit_exact(dev, golden_dir):
    import os
    gd = np.load(os.path.join(golden_dir, "greedy_decoder.npz"))
    probs = torch.from_numpy(gd["probs"])
    sizes = torch.from_numpy(gd["sizes"])
    ids, offs, counts, am = ops.greedy_decode_raw(probs.to(dev), sizes.to(dev), want_argmax=True)
    np.testing.assert_array_equal(am.cpu().numpy(), torch.max(probs, 2)[1].numpy())
    np.testing.assert_array_equal(counts.cpu().numpy(), gd["counts"])
    for i in range(probs.shape[0]):
        k = int(gd["counts"][i])
        np.testing.assert_array_equal(offs[i, :k].cpu().numpy(), gd["offsets"][i][:k])
    from ds2amd.decoder import GreedyDecoder
    dec = GreedyDecoder(orc.LABELS)
    strings, offsets = dec.decode(probs.to(dev), sizes)
    assert [s[0] for s in strings] == [str(s) for s in gd["strings"]]
    hs, ho = dec.decode(torch.from_numpy(gd["hand_probs"]).to(dev), torch.IntTensor([6]))
    assert hs[0][0] == "AA " and ho[0][0].tolist() == [1, 4, 5]
    # long utterance crossing several 64-frame chunks, strided (transposed) probs
    g = torch.Generator().manual_seed(2)
    big = torch.rand(501, 7, 30, generator=g)
    big[:, :, 0] += 0.3
    view = big.to(dev).transpose(0, 1)           # [N, T, C] non-contiguous
    s2, o2 = dec.decode(view, torch.IntTensor([501, 500, 499, 64, 63, 65, 1]))
    r2, ro2 = orc.greedy_decode(big.transpose(0, 1), [501, 500, 499, 64, 63, 65, 1])
    assert s2 == r2
    for a, b in zip(o2, ro2):
        assert a[0].tolist() == b[0].tolist()


# ---------------------------------------------------------------------------- STFT
def test_stft_vs_oracle(dev, golden_dir):
    import os
    from ds2amd.data_loader import SpectrogramParser
    gd = np.load(os.path.join(golden_dir, "cfg1_ds2.npz"))
    parser = SpectrogramParser(dict(sample_rate=16000, window_size=0.02, window_stride=0.01,
                                    window='hamming'), normalize='max_frame', device=dev)
    rng = np.random.default_rng(0)
    wavs = [gd["wav"], (rng.standard_normal(23456) * 0.3).astype(np.float32),
            np.sin(np.arange(4000) * 0.3).astype(np.float32)]
    out, frames = parser.parse_batch(wavs)
    for i, y in enumerate(wavs):
        ref = orc.spectrogram(y)
        assert int(frames[i]) == ref.shape[1]
        got = out[i, 0, :, :ref.shape[1]].cpu()
        err = (got - ref).abs().max().item()
        assert err < 2e-4, f"wav {i}: max abs err {err}"
        assert out[i, 0, :, ref.shape[1]:].abs().sum().item() == 0
    np.testing.assert_allclose(out[0, 0, :, :gd["spect"].shape[1]].cpu().numpy(), gd["spect"],
                               atol=2e-4, rtol=0)


def test_stft_spect_aug_masks_vs_oracle(dev):
    """Frequency / time bands and the 8 kHz cut zero |X| before the log and the
    'max_frame' normalisation (data_loader_aug.py:236-248): device kernel vs the oracle
    spectrogram with the same bands applied to its magnitude."""
    import random
    from ds2amd.data_loader import SpectrogramParser
    from ds2amd.spect_aug import apply_masks_np
    conf = dict(sample_rate=16000, window_size=0.02, window_stride=0.01, window='hamming',
                noise_prob=1.0, aug_prob_spect=1.0, aug_prob_8khz=0.5)
    parser = SpectrogramParser(conf, normalize='max_frame', device=dev)
    parser.spect_aug.rng = random.Random(3)
    rng = np.random.default_rng(1)
    wavs = [(rng.standard_normal(n) * 0.3).astype(np.float32) for n in (23456, 16000, 8000, 31999)]
    replay = SpectrogramParser(conf, normalize='max_frame', device=dev).spect_aug
    replay.rng = random.Random(3)
    out, frames = parser.parse_batch(wavs)
    for i, y in enumerate(wavs):
        row = replay.draw_one(161, int(frames[i]))
        mag = orc.stft_magnitude(y)
        ref = orc.normalize_max_frame(apply_masks_np(mag, row))
        got = out[i, 0, :, :ref.shape[1]].cpu()
        err = (got - ref).abs().max().item()
        assert err < 2e-4, f"wav {i} row {row}: max abs err {err}"


@pytest.mark.parametrize("sr", [8000, 11025, 22050])
@pytest.mark.parametrize("masked", [False, True])
def test_stft_other_sample_rates_vs_oracle(dev, sr, masked):
    """Sample rates other than 16 kHz (data_loader_aug.py:221-249): fewer than 161 bins
    (8 kHz: 81, 11.025 kHz: 111) take the reference's resize + mirror-fill layout, more
    (22.05 kHz: 221) are cut to 161 rows; spectrogram masks then act on the 161 rows."""
    import random
    from ds2amd.data_loader import SpectrogramParser
    from ds2amd.spect_aug import apply_masks_np
    conf = dict(sample_rate=sr, window_size=0.02, window_stride=0.01, window='hamming')
    if masked:
        conf.update(noise_prob=1.0, aug_prob_spect=1.0, aug_prob_8khz=0.5)
    parser = SpectrogramParser(conf, normalize='max_frame', device=dev)
    parser.spect_aug.rng = random.Random(5)
    replay = SpectrogramParser(conf, normalize='max_frame', device=dev).spect_aug
    replay.rng = random.Random(5)
    rng = np.random.default_rng(sr)
    wavs = [(rng.standard_normal(n) * 0.3).astype(np.float32)
            for n in (sr * 2 + 17, sr, sr // 2 + 3)]
    out, frames = parser.parse_batch(wavs, sr)
    assert out.shape[2] == 161
    for i, y in enumerate(wavs):
        mag = orc.rows161(orc.stft_magnitude(y, sr))
        if masked:
            mag = apply_masks_np(mag, replay.draw_one(161, int(frames[i])))
        ref = orc.normalize_max_frame(mag)
        assert int(frames[i]) == ref.shape[1]
        got = out[i, 0, :, :ref.shape[1]].cpu()
        err = (got - ref).abs().max().item()
        assert err < 2e-4, f"sr {sr} wav {i}: max abs err {err}"
        assert out[i, 0, :, ref.shape[1]:].abs().sum().item() == 0


@pytest.mark.parametrize("norm", ["none", "mean", "norm", "frame", "max_frame"])
@pytest.mark.parametrize("sr", [16000, 8000])
def test_stft_norm_modes_vs_oracle(dev, norm, sr):
    """Every normalize_audio mode (data_loader_aug.py:274-313; --norm, train.py:75) on the
    device against the oracle's restatement, on the 161-bin path (16 kHz) and the 8 kHz
    mirror-fill path; utterance lengths include 'frame''s sigma-50 filter (radius 200)
    reflecting over fewer frames than its radius."""
    from ds2amd.data_loader import SpectrogramParser
    conf = dict(sample_rate=sr, window_size=0.02, window_stride=0.01, window='hamming')
    parser = SpectrogramParser(conf, normalize=norm, device=dev)
    rng = np.random.default_rng(11)
    wavs = [(rng.standard_normal(n) * 0.3).astype(np.float32)
            for n in (sr * 3 + 5, sr // 2 + 7, sr // 10)]
    wavs.append(np.sin(np.arange(sr) * 0.05).astype(np.float32) * 0.5)
    out, frames = parser.parse_batch(wavs, sr)
    for i, y in enumerate(wavs):
        ref = orc.spectrogram(y, sr, normalize=norm)
        assert int(frames[i]) == ref.shape[1]
        got = out[i, 0, :, :ref.shape[1]].cpu()
        scale = max(1.0, ref.abs().max().item())
        err = (got - ref).abs().max().item()
        assert err < 2e-5 * scale + 1e-5, f"{norm} sr {sr} wav {i}: max abs err {err}"
        assert out[i, 0, :, ref.shape[1]:].abs().sum().item() == 0


def test_stft_unknown_norm_raises():
    from ds2amd.data_loader import SpectrogramParser
    p = SpectrogramParser(dict(sample_rate=16000, window_size=0.02, window_stride=0.01),
                          normalize='bogus', device='cpu')
    with pytest.raises(ValueError, match="normalize"):
        p._mode()


# ---------------------------------------------------------------------------- optimizer
def test_fused_sgd_matches_torch(dev):
    from ds2amd.optim import FlatParams, FusedSGD
    g = torch.Generator().manual_seed(4)
    shapes = [(30, 7), (13,), (5, 5, 3), (1,)]
    init = [torch.randn(s, generator=g) for s in shapes]
    ref = [torch.nn.Parameter(t.clone()) for t in init]
    opt = torch.optim.SGD(ref, lr=0.01, momentum=0.9, nesterov=True)
    mine = [torch.nn.Parameter(t.clone().to(dev)) for t in init]
    flat = FlatParams(mine, dev)
    fopt = FusedSGD(flat, lr=0.01, momentum=0.9, max_norm=1.0)
    for step in range(3):
        grads = [torch.randn(s, generator=g) * (3 if step == 1 else 0.1) for s in shapes]
        for p, gr in zip(ref, grads):
            p.grad = gr.clone()
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        opt.step()
        fopt.zero_grad()
        assert all(p.grad is None for p in mine)      # set_to_none, like torch
        for p, gr in zip(mine, grads):
            p.grad = gr.to(dev)                       # adopted into the flat buffer by step()
        fopt.step()
        for p, r in zip(mine, ref):
            _close(p, r, 1e-6, f"sgd step {step}")


def test_nan_guard_mask_and_skip(dev):
    from ds2amd.optim import FlatParams, FusedSGD
    x = torch.tensor([1.0, float('nan'), 3.0, float('nan')], device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    mask = torch.full((4,), 7, dtype=torch.uint8, device=dev)
    _lib.call("ds2_nan_guard", x.data_ptr(), 4, 1, flag.data_ptr(), mask.data_ptr(), ops._stream())
    assert flag.item() == 1 and x.tolist() == [1.0, 0.0, 3.0, 0.0]
    assert mask.tolist() == [0, 1, 0, 1]
    g = torch.tensor([5.0, 6.0, 7.0, 8.0], device=dev)
    _lib.call("ds2_zero_masked", g.data_ptr(), mask.data_ptr(), 4, flag.data_ptr(), ops._stream())
    assert g.tolist() == [5.0, 0.0, 7.0, 0.0]
    clean = torch.zeros(1, dtype=torch.int32, device=dev)       # flag 0: no-op
    g2 = torch.tensor([5.0, 6.0, 7.0, 8.0], device=dev)
    _lib.call("ds2_zero_masked", g2.data_ptr(), mask.data_ptr(), 4, clean.data_ptr(), ops._stream())
    assert g2.tolist() == [5.0, 6.0, 7.0, 8.0]
    p = torch.nn.Parameter(torch.ones(8, device=dev))
    flat = FlatParams([p], dev)
    opt = FusedSGD(flat, lr=1.0, momentum=0.9)
    p.grad.fill_(1.0)
    opt.step(skip_flag=flag)          # the C ABI's optional skip word still works
    assert torch.all(p == 1).item()


# ---------------------------------------------------------------------------- beam search
def _beam_check(dev, probs, sizes, beam, top_n=40, cutoff=1.0):
    from oracle import ctc_beam
    ids, offs, lens, scores = ops.ctc_beam_decode_raw(
        torch.from_numpy(probs).to(dev), torch.tensor(sizes, dtype=torch.int32).to(dev), beam,
        beam, cutoff_top_n=top_n, cutoff_prob=cutoff)
    ids, offs, lens, scores = ids.cpu(), offs.cpu(), lens.cpu(), scores.cpu()
    ref = ctc_beam.beam_decode(probs, sizes, beam, cutoff_top_n=top_n, cutoff_prob=cutoff)
    for n, paths in enumerate(ref):
        for p in range(beam):
            if p >= len(paths):
                assert int(lens[n, p]) == 0
                continue
            s, rid, rts = paths[p]
            k = int(lens[n, p])
            assert ids[n, p, :k].tolist() == rid, (n, p)
            assert offs[n, p, :k].tolist() == rts, (n, p)
            assert abs(float(scores[n, p]) - s) <= 1e-5 * max(1.0, abs(s)), (n, p)


@pytest.mark.parametrize("beam,top_n,cutoff,c", [(8, 40, 1.0, 30), (4, 5, 1.0, 30),
                                                 (6, 40, 0.95, 30), (1, 40, 1.0, 30),
                                                 (100, 40, 1.0, 29), (128, 40, 1.0, 32),
                                                 (100, 10, 0.99, 29), (33, 40, 1.0, 29)])
def test_ctc_beam_vs_oracle(dev, beam, top_n, cutoff, c):
    """ds2_ctc_beam_decode == oracle/ctc_beam.py (prefix beam search, no LM): ids, char
    frames and lengths bit-exact for every returned beam, scores to 1e-5 rel.  Beams
    above 32 (the reference default is 100, decoder.py:89) take the 128-entry kernel."""
    g = np.random.default_rng(beam * 10 + top_n)
    n, t = 5, 37
    logits = g.standard_normal((n, t, c)).astype(np.float32) * 3
    logits[:, :, 0] += 1.5                                  # blank-heavy, like a trained model
    probs = np.exp(logits - logits.max(-1, keepdims=True))
    probs = (probs / probs.sum(-1, keepdims=True)).astype(np.float32)
    _beam_check(dev, probs, [37, 30, 1, 0, 22], beam, top_n, cutoff)


def test_ctc_beam_hand_case_and_decoder(dev):
    from ds2amd.decoder import BeamCTCDecoder
    probs = np.array([[[0.6, 0.4], [0.6, 0.4]]], np.float32)
    _beam_check(dev, probs, [2], 4)
    dec = BeamCTCDecoder("_a", beam_width=2)
    strings, offsets = dec.decode(torch.from_numpy(probs).to(dev), torch.IntTensor([2]))
    assert strings == [["a", ""]]
    assert offsets[0][0].tolist() == [0]
    # the reference's constructor defaults (beam_width=100) over its own 29 labels
    dec = BeamCTCDecoder(orc.LABELS)
    assert dec.beam_width == 100
    g = np.random.default_rng(5)
    logits = g.standard_normal((2, 25, len(orc.LABELS))).astype(np.float32) * 3
    logits[:, :, 0] += 1.5
    p = np.exp(logits - logits.max(-1, keepdims=True))
    p = (p / p.sum(-1, keepdims=True)).astype(np.float32)
    strings, _ = dec.decode(torch.from_numpy(p).to(dev), torch.IntTensor([25, 17]))
    from oracle import ctc_beam
    ref = ctc_beam.beam_decode(p, [25, 17], 100, cutoff_top_n=40, cutoff_prob=1.0)
    for n, paths in enumerate(ref):
        assert len(strings[n]) == 100
        for q, (_, rid, _) in enumerate(paths):
            assert strings[n][q] == ''.join(orc.LABELS[i] for i in rid), (n, q)


def _spelled(text, g, noise, peak=5.0, blank_bias=1.0):
    labels = orc.LABELS
    frames, prev = [], None
    for ch in text:
        if ch == prev:
            frames.append(0)
        frames += [labels.index(ch), 0]
        prev = ch
    logits = g.standard_normal((len(frames), len(labels))).astype(np.float32) * noise
    logits[:, 0] += blank_bias
    logits[np.arange(len(frames)), frames] += peak
    p = np.exp(logits - logits.max(-1, keepdims=True))
    return (p / p.sum(-1, keepdims=True)).astype(np.float32)


@pytest.mark.parametrize("beam,top_n,cutoff,alpha,beta,noise",
                         [(8, 40, 1.0, 0.8, 1.0, 1.5), (4, 40, 1.0, 2.0, -0.5, 2.0),
                          (16, 10, 0.99, 0.8, 1.0, 2.0), (32, 40, 1.0, 0.3, 2.0, 2.5),
                          (100, 40, 1.0, 0.8, 1.0, 2.0), (33, 8, 1.0, 1.2, 0.5, 3.0)])
def test_ctc_beam_lm_vs_oracle(dev, beam, top_n, cutoff, alpha, beta, noise):
    """ds2_ctc_beam_decode_lm (BeamCTCDecoder with lm_path) == oracle/ctc_beam_lm.py
    (ctcdecode's KenLM Scorer semantics restated; ctcdecode itself is absent, parity with
    it unpinned) on the committed 3-gram tests/golden/tiny_lm.arpa: ids, char frames and
    lengths of every returned beam bit-exact, scores to 1e-5 rel.  Noisy spelled
    sentences (word boundaries, back-off chains, words outside the vocabulary), sizes 0
    and 1, both kernel sizes (beams <= 32 and the 128-entry kernel)."""
    from oracle import ctc_beam_lm as obl
    from ds2amd.lm import ArpaScorer
    path = os.path.join(os.path.dirname(__file__), "golden", "tiny_lm.arpa")
    labels = orc.LABELS
    g = np.random.default_rng(beam * 7 + top_n)
    texts = ["THE CAT SAT ", "I DON'T NO ", "AND THEY SAT ON A HAT", "CATS IN THEN"]
    ps = [_spelled(s, g, noise) for s in texts]
    t = max(p.shape[0] for p in ps)
    probs = np.full((len(ps) + 2, t, len(labels)), 1.0 / len(labels), np.float32)
    for i, p in enumerate(ps):
        probs[i, :p.shape[0]] = p
    sizes = [p.shape[0] for p in ps] + [0, 1]
    scorer = ArpaScorer(path, labels, alpha, beta, device=dev)
    ids, offs, lens, scores = ops.ctc_beam_decode_lm_raw(
        torch.from_numpy(probs).to(dev), torch.tensor(sizes, dtype=torch.int32).to(dev), beam,
        beam, scorer, cutoff_top_n=top_n, cutoff_prob=cutoff)
    ids, offs, lens, scores = ids.cpu(), offs.cpu(), lens.cpu(), scores.cpu()
    lm = obl.ArpaLM(path)
    ref = obl.beam_decode_lm(probs, sizes, beam, lm, labels, alpha, beta, cutoff_top_n=top_n,
                             cutoff_prob=cutoff)
    for n, paths in enumerate(ref):
        for p in range(beam):
            if p >= len(paths):
                assert int(lens[n, p]) == 0
                continue
            s, rid, rts = paths[p]
            k = int(lens[n, p])
            assert ids[n, p, :k].tolist() == rid, (n, p, ids[n, p, :k].tolist(), rid)
            assert offs[n, p, :k].tolist() == rts, (n, p)
            assert abs(float(scores[n, p]) - s) <= 1e-5 * max(1.0, abs(s)), (n, p)
    # the decoder front end: lm_path -> the same best strings
    from ds2amd.decoder import BeamCTCDecoder
    dec = BeamCTCDecoder(labels, lm_path=path, alpha=alpha, beta=beta, cutoff_top_n=top_n,
                         cutoff_prob=cutoff, beam_width=beam)
    strings, _ = dec.decode(torch.from_numpy(probs).to(dev), torch.tensor(sizes, dtype=torch.int32))
    for n, paths in enumerate(ref):   # (a beam pruned empty returns '' everywhere)
        assert strings[n][0] == (''.join(labels[i] for i in paths[0][1]) if paths else '')


@pytest.mark.parametrize("order,beam", [(1, 16), (2, 8), (5, 16), (6, 100)])
def test_ctc_beam_lm_orders_vs_oracle(dev, order, beam, tmp_path):
    """The LM search with models of every order the kernel takes (1..6: no history, the
    <s>-padded histories up to five words, back-off chains up to six lookups), generated by
    tests/golden/make_lm_fixture.build(order=...), against oracle/ctc_beam_lm.py."""
    import importlib.util
    from oracle import ctc_beam_lm as obl
    from ds2amd.lm import ArpaScorer
    spec = importlib.util.spec_from_file_location(
        "make_lm_fixture", os.path.join(os.path.dirname(__file__), "golden", "make_lm_fixture.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    path = str(tmp_path / f"lm{order}.arpa")
    with open(path, "w", encoding="utf-8") as f:
        f.write(mk.build(seed=order, order=order, top=60))
    labels = orc.LABELS
    g = np.random.default_rng(order)
    texts = ["THE CAT SAT ON A HAT", "I DON'T NO THEN ", "CATS AND DOG TOO"]
    ps = [_spelled(s, g, 2.0) for s in texts]
    t = max(p.shape[0] for p in ps)
    probs = np.full((len(ps), t, len(labels)), 1.0 / len(labels), np.float32)
    for i, p in enumerate(ps):
        probs[i, :p.shape[0]] = p
    sizes = [p.shape[0] for p in ps]
    scorer = ArpaScorer(path, labels, 1.1, 0.7, device=dev)
    assert scorer.order == order
    ids, offs, lens, scores = ops.ctc_beam_decode_lm_raw(
        torch.from_numpy(probs).to(dev), torch.tensor(sizes, dtype=torch.int32).to(dev), beam,
        beam, scorer)
    ids, offs, lens, scores = ids.cpu(), offs.cpu(), lens.cpu(), scores.cpu()
    ref = obl.beam_decode_lm(probs, sizes, beam, obl.ArpaLM(path), labels, 1.1, 0.7)
    for n, paths in enumerate(ref):
        for p in range(beam):
            if p >= len(paths):
                assert int(lens[n, p]) == 0
                continue
            s_, rid, rts = paths[p]
            k = int(lens[n, p])
            assert ids[n, p, :k].tolist() == rid, (n, p)
            assert offs[n, p, :k].tolist() == rts, (n, p)
            assert abs(float(scores[n, p]) - s_) <= 1e-5 * max(1.0, abs(s_)), (n, p)


@pytest.mark.parametrize("noise,beam", [(2.0, 100), (3.0, 100), (3.0, 32)])
def test_ctc_beam_trie_revival_vs_oracle(dev, noise, beam):
    """Trie-node revival (ctcdecode path_trie.cpp get_path_trie / remove): a pruned prefix
    kept in the trie by a descendant in the beam is revived by an extension onto it (its
    node, char frame and dictionary state kept) rather than created again.  Noisy spelled
    sentences where the oracle revives prefixes (counted), with and without the LM: the
    device search equals oracle/ctc_beam.py / ctc_beam_lm.py bit-exactly (ids, frames) and
    every returned beam holds distinct strings."""
    from oracle import ctc_beam, ctc_beam_lm as obl
    from ds2amd.lm import ArpaScorer
    labels = orc.LABELS
    g = np.random.default_rng(11)
    ps = [_spelled(s, g, noise) for s in ["THE CAT SAT ON A HAT", "I DON'T NO THEN ",
                                          "AND THEY SAT ON A CAT", "CATS IN THEN TOO"]]
    t = max(p.shape[0] for p in ps)
    probs = np.full((len(ps), t, len(labels)), 1.0 / len(labels), np.float32)
    for i, p in enumerate(ps):
        probs[i, :p.shape[0]] = p
    sizes = [p.shape[0] for p in ps]
    ctc_beam.STATS["revived"] = 0
    _beam_check(dev, probs, sizes, beam)
    path = os.path.join(os.path.dirname(__file__), "golden", "tiny_lm.arpa")
    scorer = ArpaScorer(path, labels, 0.8, 1.0, device=dev)
    ids, offs, lens, scores = ops.ctc_beam_decode_lm_raw(
        torch.from_numpy(probs).to(dev), torch.tensor(sizes, dtype=torch.int32).to(dev), beam,
        beam, scorer)
    ids, offs, lens = ids.cpu(), offs.cpu(), lens.cpu()
    ref = obl.beam_decode_lm(probs, sizes, beam, obl.ArpaLM(path), labels, 0.8, 1.0)
    assert ctc_beam.STATS["revived"] > 0
    for n, paths in enumerate(ref):
        got = []
        for p in range(len(paths)):
            k = int(lens[n, p])
            got.append(tuple(ids[n, p, :k].tolist()))
            assert list(got[-1]) == paths[p][1], (n, p)
            assert offs[n, p, :k].tolist() == paths[p][2], (n, p)
        assert len(set(got)) == len(got)


# ---------------------------------------------------------------------------- CER / WER
def test_edit_distance_vs_reference_semantics(dev):
    """ds2_edit_distance == get_cer_wer (data/utils.py:47-57) with Decoder.wer/.cer's
    Levenshtein on the same strings: random id strings with runs of spaces, leading /
    trailing spaces, empty sequences, identical pairs and long sequences."""
    from ds2amd.decoder import Decoder
    from ds2amd.trainer import get_cer_wer
    labels = orc.LABELS
    space = labels.index(' ')
    dec = Decoder(labels)
    g = np.random.default_rng(17)
    a_rows, b_rows = [], []
    for i in range(40):
        la = int(g.integers(0, 120)) if i % 10 else 0
        lb = int(g.integers(0, 90)) if i % 7 else 0
        alphabet = [space, space, 1, 2, 3, 4, 5] if i % 3 == 0 else list(range(1, len(labels)))
        a_rows.append([int(alphabet[k]) for k in g.integers(0, len(alphabet), la)])
        b_rows.append([int(alphabet[k]) for k in g.integers(0, len(alphabet), lb)])
    a_rows.append(list(range(1, 29)) * 40)          # 1120 ids
    b_rows.append(list(range(1, 29)) * 35)
    a_rows.append([5, space, 6, space, space, 5])   # identical after strip / split
    b_rows.append([space, 5, space, 6, space, 5, space])
    # reference lengths on both sides of the register-row DP's 64-column chunks (1-4 chunks
    # in registers below 256 columns, the LDS-row DP from 256 on)
    for lb in (63, 64, 127, 128, 191, 192, 255, 256):
        a_rows.append([int(k) for k in g.integers(1, space, 300)])   # no spaces: n = lb
        b_rows.append([int(k) for k in g.integers(1, space, lb)])
    n = len(a_rows)
    width = max(len(r) for r in a_rows)
    a = torch.zeros(n, width, dtype=torch.int32)
    for i, r in enumerate(a_rows):
        a[i, :len(r)] = torch.tensor(r, dtype=torch.int32)
    a_lens = torch.tensor([len(r) for r in a_rows], dtype=torch.int32)
    b = torch.tensor([x for r in b_rows for x in r], dtype=torch.int32)
    b_lens = torch.tensor([len(r) for r in b_rows], dtype=torch.int32)
    out, err = ops.edit_distance_raw(a.to(dev), a_lens, b, b_lens, space)
    out = out.cpu()
    assert int(err.item()) == 0
    to_s = lambda r: ''.join(labels[k] for k in r)
    for i in range(n):
        wer, cer, wref, cref = get_cer_wer(dec, to_s(a_rows[i]), to_s(b_rows[i]))
        assert out[i].tolist() == [wer, cer, int(wref), int(cref)], i


# ---------------------------------------------------------------------------- colsum
@pytest.mark.parametrize("rows,cols,ld,off", [(16032, 2400, 4800, 0), (16032, 2400, 4800, 2400),
                                              (37, 5, 7, 1), (1000, 260, 260, 0)])
@pytest.mark.parametrize("accumulate", [0, 1])
def test_colsum(dev, rows, cols, ld, off, accumulate):
    """ds2_colsum (bias gradients): vector and scalar paths vs a float64 reference."""
    g = torch.Generator().manual_seed(rows + cols + off)
    x = torch.randn(rows, ld, generator=g)
    out0 = torch.randn(cols, generator=g)
    ref = x[:, off:off + cols].double().sum(0) + (out0.double() if accumulate else 0.0)
    out = out0.to(dev).clone()
    ops.colsum(x.to(dev), rows, cols, ld, out, accumulate=bool(accumulate), off=off)
    _close(out, ref, 1e-6, "colsum")


@pytest.mark.parametrize("cell,nd", [("gru", 1), ("gru", 2), ("lstm", 1), ("lstm", 2),
                                     ("rnn", 1), ("rnn", 2)])
def test_rnn_param_grads_bf16_shared_copies(dev, cell, nd):
    """the cfg4 backward's bf16 parameter gradients from operand copies made ONCE per
    layer (ops._rnn_param_grads_bf16: dW_ih, dW_hh with the per-direction one-step k shift, dX
    through the concatenated W_ih, bias sums) against the per-GEMM bf16 conversions of
    sgemm(bf16=True) -- the same bf16 products, only the fp32 summation order (tile plans)
    differs: 1e-5 of each gradient's max.  N = 16, every size a multiple of 8 (the fast
    path's condition)."""
    torch.manual_seed(5)
    t, n, inp, h = 9, 16, 64, 32
    g = {"gru": 3 * h, "lstm": 4 * h, "rnn": h}[cell]
    x = torch.randn(t, n, inp, device=dev)
    h_all = torch.randn(t, n, nd, h, device=dev)
    dgx = torch.randn(t, n, nd, g, device=dev)
    dgh = dgx if cell == "lstm" else torch.randn(t, n, nd, g, device=dev)
    if cell == "gru":   # the kernels store the same r, z columns in both
        dgh[..., :2 * h] = dgx[..., :2 * h]
    weights = []
    for _ in range(nd):
        weights += [torch.randn(g, inp, device=dev), torch.randn(g, h, device=dev),
                    torch.randn(g, device=dev), torch.randn(g, device=dev)]
    dx_f, gr_f = ops._rnn_param_grads(x, h_all, dgx, dgh, weights, nd, g, True, bf16=True)
    dx_p, gr_p = ops._rnn_param_grads(x, h_all, dgx, dgh, weights, nd, g, True, bf16=True,
                                      shared_bf16=False)
    torch.cuda.synchronize()
    _close(dx_f, dx_p, 1e-5, "dx")
    names = ["dw_ih", "dw_hh", "db_ih", "db_hh"]
    for i, (a, b) in enumerate(zip(gr_f, gr_p)):
        _close(a, b, 1e-5, f"{names[i % 4]} dir {i // 4}")
    # and both really are bf16 products: the fp32 path differs by far more than 1e-5
    _, gr_32 = ops._rnn_param_grads(x, h_all, dgx, dgh, weights, nd, g, True, bf16=False)
    d = (gr_32[0] - gr_f[0]).abs().max().item() / gr_32[0].abs().max().item()
    assert d > 1e-4, d


@pytest.mark.parametrize("bwd", ["h3", "x6"])
@pytest.mark.parametrize("n,h,bidir", [(32, 800, True), (7, 48, False), (20, 256, True)])
def test_gru_bwd_column_maxima(dev, n, h, bidir, bwd, monkeypatch):
    """ds2_gru_bwd_bias_amax: the column maxima of dgx / dgh the fp16x3 GEMMs scale by, kept
    by the fp16x3 backward recurrence as it runs (bwd='h3') or by a column pass after the
    bf16x6 one (DS2_GRU_H3_BWD=0): bit-exact against torch's amax of the gradients the layer
    handed to its GEMMs."""
    monkeypatch.setenv("DS2_GRU_H3_BWD", "1" if bwd == "h3" else "0")
    nd = 2 if bidir else 1
    seen = {}
    orig = ops._rnn_param_grads

    def spy(x, h_all, dgx, dgh, weights, nd_, g, need_dx, bf16=False, pre=None, dbias=None, **kw):
        seen["dgx"], seen["dgh"], seen["col"] = dgx.clone(), dgh.clone(), kw.get("col_amax")
        return orig(x, h_all, dgx, dgh, weights, nd_, g, need_dx, bf16, pre, dbias, **kw)

    monkeypatch.setattr(ops, "_rnn_param_grads", spy)
    _gru_run(dev, n, 29, 40, h, nd, h + n, [{}], monkeypatch)
    col = seen["col"]
    assert col is not None
    g = nd * 3 * h
    ref_x = seen["dgx"].view(-1, g).abs().amax(0).contiguous().view(torch.int32)
    ref_h = seen["dgh"].view(-1, g).abs().amax(0).contiguous().view(torch.int32)
    assert torch.equal(col[:g], ref_x)
    assert torch.equal(col[g:], ref_h)


@pytest.mark.parametrize("n,h,nd", [(64, 1024, 2), (64, 1024, 1), (32, 800, 2), (16, 256, 1)])
def test_lstm_half_grid_covers_its_fallback(dev, n, h, nd):
    """ds2_lstm_bwd_half_grid budgets the co-residency guard for ds2_lstm_bwd_half, which falls
    back to ds2_lstm_bwd (16-sample tiles, up to twice the workgroups) when its own kernel
    declines: the reported grid must cover both, as ds2_gru_bwd_grid covers the
    XCD-local kernel and its fallbacks."""
    half = ops.persistent_bwd_grid("lstm_half", n, h, nd)
    full = ops.persistent_bwd_grid("lstm", n, h, nd)
    assert half >= full
