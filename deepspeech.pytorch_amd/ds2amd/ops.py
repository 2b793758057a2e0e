"""Device ops over the libds2hip C ABI, plus their autograd wrappers.

Every function here hands raw device pointers to a HIP kernel through
``_lib.call``; torch supplies only memory (caching allocator), the current HIP
stream and autograd bookkeeping.  Inputs must be CUDA (HIP) float32/int32
tensors; there is no CPU path (the CPU restatement lives in ``oracle/`` and is
used only by the tests and the bench's cpu_baseline leg).
"""
from __future__ import annotations

from typing import Optional, Tuple

import os
import numpy as np
import torch

from . import _lib

_F32 = torch.float32
_I32 = torch.int32


# ----------------------------------------------------------------------------
# plumbing
def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _need(t: torch.Tensor, name: str, dtype=_F32) -> torch.Tensor:
    if not t.is_cuda:
        raise _lib.Ds2Error(f"{name}: expected a device tensor (got {t.device}); "
                            "the ds2amd product path runs only on the GPU")
    if t.dtype != dtype:
        raise _lib.Ds2Error(f"{name}: expected {dtype}, got {t.dtype}")
    return t.contiguous()


def _ws(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


# Hand-off status of the persistent recurrence kernels (ds2hip.h err_out): one device word per
# device, OR-ed by every ds2_gru_* / ds2_lstm_* launch and never cleared by the library.  It is
# read only where the host synchronises anyway (Trainer.poll_status / check_rnn_status), so a
# hand-off timeout raises Ds2Error instead of turning into a silently NaN-zeroed step.
RNN_ERR_HANDOFF_TIMEOUT = 1
_RNN_STATUS = {}


def rnn_status_word(device) -> torch.Tensor:
    device = torch.device(device)
    if device.index is None:
        device = torch.device(device.type, torch.cuda.current_device())
    w = _RNN_STATUS.get(device)
    if w is None:
        w = torch.zeros(1, dtype=_I32, device=device)
        _RNN_STATUS[device] = w
    return w


def rnn_status_error(value: int) -> Optional[str]:
    if value == 0:
        return None
    what = []
    if value & RNN_ERR_HANDOFF_TIMEOUT:
        what.append("hand-off timeout (a workgroup of a persistent GRU/LSTM kernel waited past "
                    "its spin bound; outputs from that step on are NaN)")
    if value & ~RNN_ERR_HANDOFF_TIMEOUT:
        what.append(f"unknown status bits 0x{value & ~RNN_ERR_HANDOFF_TIMEOUT:x}")
    return "recurrence kernel failure: " + "; ".join(what)


def check_rnn_status(device=None, reset: bool = True) -> None:
    """Synchronising read of the device status word; raises Ds2Error if any recurrence launch
    since the last reset reported a failure."""
    w = rnn_status_word(device if device is not None else torch.device("cuda"))
    v = int(w.item())
    if reset and v:
        w.zero_()
    msg = rnn_status_error(v)
    if msg is not None:
        raise _lib.Ds2Error(msg)


# ----------------------------------------------------------------------------
# raw ops
def sgemm(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor, *, m: int, n: int, k: int,
          trans_a: bool = False, trans_b: bool = False, lda: int, ldb: int, ldc: int,
          alpha: float = 1.0, beta: float = 0.0, bias: Optional[torch.Tensor] = None,
          a_off: int = 0, b_off: int = 0, c_off: int = 0, bf16: bool = False,
          a_amax: Optional[torch.Tensor] = None, b_amax: Optional[torch.Tensor] = None
          ) -> torch.Tensor:
    """C = alpha*op(A)@op(B) + beta*C (+bias) on raw row-major storage.

    ``*_off`` are element offsets into the (contiguous) storage of a/b/c.  ``bf16``: the
    operands are rounded to bf16 and multiplied on the bf16 MFMA (fp32 accumulation,
    ds2_sgemm_bf16_ws) -- the opt-in precision of BASELINE cfg4's RNN GEMMs.
    ``a_amax`` / ``b_amax``: int32 tensors holding the float bits of max |op(A)[m, :]| /
    max |op(B)[:, n]| (ds2_amax; an upper bound is valid): the fp16x3 kernel's row scales,
    shared between GEMMs instead of recomputed by each (ds2_sgemm_amax_ws).
    """
    es = 4
    if (a_amax is not None or b_amax is not None) and not bf16:
        nbytes = _lib.size("ds2_sgemm_workspace_size", m, n, k, 1)
        ws = _ws(nbytes, c.device) if nbytes > 0 else None
        _lib.call("ds2_sgemm_amax_ws", int(trans_a), int(trans_b), m, n, k, float(alpha),
                  a.data_ptr() + es * a_off, lda, b.data_ptr() + es * b_off, ldb, float(beta),
                  c.data_ptr() + es * c_off, ldc, _p(bias), _p(a_amax), _p(b_amax), _p(ws),
                  0 if ws is None else ws.numel(), _stream())
        return c
    # ds2_bgemm_nt takes bf16 copies of < 2 GiB each: larger operands stay on the
    # staged-rounding kernel (ds2_sgemm_bf16_ws), which has no such limit
    if (bf16 and k % 8 == 0 and k > 0 and m > 0 and n > 0 and 2 * m * k < 2**31
            and 2 * n * k < 2**31):
        return _sgemm_bf16_bgemm(a, b, c, m, n, k, trans_a, trans_b, lda, ldb, ldc, alpha, beta,
                                 bias, a_off, b_off, c_off)
    fn = "ds2_sgemm_bf16" if bf16 else "ds2_sgemm"
    nbytes = _lib.size(fn + "_workspace_size", m, n, k, 1)
    ws = _ws(nbytes, c.device) if nbytes > 0 else None
    _lib.call(fn + "_ws", int(trans_a), int(trans_b), m, n, k, float(alpha),
              a.data_ptr() + es * a_off, lda, 0, b.data_ptr() + es * b_off, ldb, 0,
              float(beta), c.data_ptr() + es * c_off, ldc, 0, 1, _p(bias), _p(ws),
              0 if ws is None else ws.numel(), _stream())
    return c


def h3_enabled() -> bool:
    """The fp16x3 GEMM kernel is in use (the default; DS2_GEMM_H3=0 or DS2_GEMM_X6=0 turn it
    off -- the library reads the same variables per call)."""
    return os.environ.get("DS2_GEMM_H3", "1")[:1] != "0" and \
        os.environ.get("DS2_GEMM_X6", "1")[:1] != "0"


def amax(x: torch.Tensor, rows: int, cols: int, ld: int, off: int = 0, want_rows: bool = True,
         want_cols: bool = True):
    """(row maxima, column maxima) of |x| over the [rows][cols] matrix at element offset
    ``off`` of x's storage (leading dimension ld) as int32 float bits (ds2_amax, one pass);
    None for a part not asked for, or for both when the operand is not float4-aligned."""
    ptr = x.data_ptr() + 4 * off
    if ptr % 16 or cols % 4 or ld % 4 or rows <= 0 or cols <= 0:
        return None, None
    r = torch.empty(rows, dtype=_I32, device=x.device) if want_rows else None
    c = torch.empty(cols, dtype=_I32, device=x.device) if want_cols else None
    _lib.call("ds2_amax", ptr, rows, cols, ld, _p(r), _p(c), _stream())
    return r, c


_ONE_BITS = {}


def unit_bound(n: int, device) -> torch.Tensor:
    """n float bits of 1.0: the fp16x3 scale bound of tanh-bounded operands (the recurrent
    states h, |h| < 1)."""
    key = (n, str(device))
    t = _ONE_BITS.get(key)
    if t is None:
        t = torch.full((n,), 0x3F800000, dtype=_I32, device=device)
        _ONE_BITS[key] = t
    return t


def _sgemm_bf16_bgemm(a, b, c, m, n, k, trans_a, trans_b, lda, ldb, ldc, alpha, beta, bias,
                      a_off, b_off, c_off):
    """The bf16 RNN GEMMs (BASELINE cfg4) on ds2_bgemm_nt: both operands rounded to bf16 into
    k-contiguous copies (A -> [m][k], B -> [n][k]; ds2_cvt_bf16, transposing where the operand
    is m- or n-contiguous), then the bf16 MFMA GEMM.  Same rounding (RNE) and products as
    ds2_sgemm_bf16_ws; only the fp32 summation order differs."""
    dev = c.device
    cp = a.data_ptr() + 4 * a_off
    ab = torch.empty(m, k, device=dev, dtype=torch.bfloat16)
    if trans_a:   # A stored [k][m]
        _lib.call("ds2_cvt_bf16", cp, k, m, lda, ab.data_ptr(), k, 1, _stream())
    else:
        _lib.call("ds2_cvt_bf16", cp, m, k, lda, ab.data_ptr(), k, 0, _stream())
    bp = b.data_ptr() + 4 * b_off
    bb = torch.empty(n, k, device=dev, dtype=torch.bfloat16)
    if trans_b:   # B stored [n][k]
        _lib.call("ds2_cvt_bf16", bp, n, k, ldb, bb.data_ptr(), k, 0, _stream())
    else:         # B stored [k][n]
        _lib.call("ds2_cvt_bf16", bp, k, n, ldb, bb.data_ptr(), k, 1, _stream())
    nbytes = _lib.size("ds2_bgemm_workspace_size", m, n, k)
    ws = _ws(nbytes, dev) if nbytes > 0 else None
    _lib.call("ds2_bgemm_nt", m, n, k, float(alpha), ab.data_ptr(), k, bb.data_ptr(), k,
              float(beta), c.data_ptr() + 4 * c_off, ldc, _p(bias), _p(ws),
              0 if ws is None else ws.numel(), _stream())
    return c


def to_bf16(x: torch.Tensor, transpose: bool = False,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 [rows, cols] (row-major, contiguous rows) -> bf16 (round to nearest even) on the
    device (ds2_cvt_bf16), as is or transposed ([cols, rows]): the k-contiguous bf16 copy an
    operand of ds2_bgemm_nt needs."""
    if not x.is_cuda or x.dtype != _F32 or x.dim() != 2 or x.stride(1) != 1:
        raise _lib.Ds2Error("to_bf16: expected a row-major float32 device matrix")
    rows, cols = x.shape
    shape = (cols, rows) if transpose else (rows, cols)
    if out is None:
        out = torch.empty(shape, device=x.device, dtype=torch.bfloat16)
    _lib.call("ds2_cvt_bf16", x.data_ptr(), rows, cols, x.stride(0), out.data_ptr(),
              out.stride(0), int(transpose), _stream())
    return out


def bgemm_nt(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor, *, alpha: float = 1.0,
             beta: float = 0.0, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """c[m, n] (fp32) = alpha * a[m, k] @ b[n, k]^T + beta * c (+ bias): bf16 operands
    (k-contiguous), bf16 MFMA, fp32 accumulation (ds2_bgemm_nt, csrc/bgemm.hip)."""
    for t in (a, b):
        if not t.is_cuda or t.dtype != torch.bfloat16 or t.dim() != 2 or t.stride(1) != 1:
            raise _lib.Ds2Error("bgemm_nt: expected row-major bf16 device matrices")
    m, k = a.shape
    n = b.shape[0]
    if b.shape[1] != k or tuple(c.shape) != (m, n) or c.dtype != _F32:
        raise _lib.Ds2Error(f"bgemm_nt: shapes a {tuple(a.shape)} b {tuple(b.shape)} c {tuple(c.shape)}")
    nbytes = _lib.size("ds2_bgemm_workspace_size", m, n, k)
    ws = _ws(nbytes, c.device) if nbytes > 0 else None
    _lib.call("ds2_bgemm_nt", m, n, k, float(alpha), a.data_ptr(), a.stride(0), b.data_ptr(),
              b.stride(0), float(beta), c.data_ptr(), c.stride(0), _p(bias), _p(ws),
              0 if ws is None else ws.numel(), _stream())
    return c


def matmul_nt(x2d: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x2d[M,K] @ w[N,K]^T (+bias) -> [M,N] (nn.Linear forward)."""
    m, k = x2d.shape
    n = w.shape[0]
    if out is None:
        out = torch.empty(m, n, device=x2d.device, dtype=_F32)
    return sgemm(x2d, w, out, m=m, n=n, k=k, trans_b=True, lda=k, ldb=k, ldc=n, bias=bias)


# Gradient slots (optim.FlatParams): a registered parameter whose .grad is None gets its
# gradient written straight into its slice of the flat gradient buffer; autograd then
# adopts that view as p.grad (no accumulate kernel, no copy).  With p.grad already set
# (backward without zero_grad) a fresh tensor is returned and autograd accumulates.
_GRAD_SLOTS = {}


def register_grad_slot(param, flat_grad, offset):
    _GRAD_SLOTS[param.data_ptr()] = (flat_grad, int(offset), tuple(param.shape))


def grad_like(param):
    slot = _GRAD_SLOTS.get(param.data_ptr())
    if slot is not None and param.grad is None and slot[2] == tuple(param.shape):
        buf, off, shape = slot
        return buf.narrow(0, off, param.numel()).view(shape)
    return torch.empty_like(param)


def conv_out_shape(h: int, w: int, kh: int, kw: int, sh: int, sw: int, ph: int, pw: int):
    return (h + 2 * ph - kh) // sh + 1, (w + 2 * pw - kw) // sw + 1


def conv2d_fwd(x, weight, bias, stride, padding, out_lens=None):
    x = _need(x, "conv2d.x")
    weight = _need(weight, "conv2d.weight")
    n, ci, h, w = x.shape
    co, _, kh, kw = weight.shape
    ho, wo = conv_out_shape(h, w, kh, kw, stride[0], stride[1], padding[0], padding[1])
    y = torch.empty(n, co, ho, wo, device=x.device, dtype=_F32)
    dims = (n, ci, h, w, co, kh, kw, stride[0], stride[1], padding[0], padding[1])
    ws = _ws(_lib.size("ds2_conv2d_workspace_size", *dims), x.device)
    _lib.call("ds2_conv2d_fwd", x.data_ptr(), weight.data_ptr(),
              _p(None if bias is None else _need(bias, "conv2d.bias")), y.data_ptr(), *dims,
              _p(out_lens), ws.data_ptr(), ws.numel(), _stream())
    return y


def conv2d_dgrad(dy, weight, x_shape, stride, padding):
    dy = _need(dy, "conv2d.dy")
    n, ci, h, w = x_shape
    co, _, kh, kw = weight.shape
    dx = torch.empty(n, ci, h, w, device=dy.device, dtype=_F32)
    dims = (n, ci, h, w, co, kh, kw, stride[0], stride[1], padding[0], padding[1])
    ws = _ws(_lib.size("ds2_conv2d_workspace_size", *dims), dy.device)
    _lib.call("ds2_conv2d_dgrad", dy.data_ptr(), weight.data_ptr(), dx.data_ptr(), *dims,
              ws.data_ptr(), ws.numel(), _stream())
    return dx


def conv2d_wgrad(dy, x, w_shape, stride, padding, with_bias: bool, out_dw=None, out_db=None):
    dy = _need(dy, "conv2d.dy")
    x = _need(x, "conv2d.x")
    n, ci, h, w = x.shape
    co, _, kh, kw = w_shape
    dw = out_dw if out_dw is not None else torch.empty(w_shape, device=x.device, dtype=_F32)
    db = None
    if with_bias:
        db = out_db if out_db is not None else torch.empty(co, device=x.device, dtype=_F32)
    dims = (n, ci, h, w, co, kh, kw, stride[0], stride[1], padding[0], padding[1])
    nbytes = _lib.size("ds2_conv2d_wgrad_workspace_size", *dims)
    ws = _ws(nbytes, x.device)
    _lib.call("ds2_conv2d_wgrad", dy.data_ptr(), x.data_ptr(), dw.data_ptr(), _p(db), *dims,
              ws.data_ptr(), ws.numel(), _stream())
    return dw, db


def bn_stats(x, outer, c, inner, eps, momentum, running_mean, running_var, training):
    mean = torch.empty(c, device=x.device, dtype=_F32)
    invstd = torch.empty(c, device=x.device, dtype=_F32)
    if training:
        ws = _ws(_lib.size("ds2_bn_workspace_size", outer, c, inner), x.device)
        _lib.call("ds2_bn_train_stats", x.data_ptr(), outer, c, inner, float(eps), float(momentum),
                  mean.data_ptr(), invstd.data_ptr(), _p(running_mean), _p(running_var),
                  ws.data_ptr(), ws.numel(), _stream())
    else:
        _lib.call("ds2_bn_eval_stats", running_mean.data_ptr(), running_var.data_ptr(), c,
                  float(eps), mean.data_ptr(), invstd.data_ptr(), _stream())
    return mean, invstd


def bn_apply(x, outer, c, inner, mean, invstd, gamma, beta):
    y = torch.empty_like(x)
    _lib.call("ds2_bn_apply", x.data_ptr(), outer, c, inner, mean.data_ptr(), invstd.data_ptr(),
              gamma.data_ptr(), beta.data_ptr(), y.data_ptr(), _stream())
    return y


# fp16x3 GEMM scales written by the kernel that produced an operand (ds2_bn_apply_amax), handed
# to the GEMMs that read it next (the input projection: row maxima; dW_ih: column maxima).  An
# entry holds the operand itself, so its storage cannot be reused while the entry lives, and is
# valid only for the same storage, element count and version (views share the base's version
# counter); the consumer pops it.  A few entries at most: an unconsumed one is dropped.
_OPERAND_AMAX = []


def _tag_amax(y, rows, cols, rmax, cmax):
    _OPERAND_AMAX.append((y, y.data_ptr(), rows, cols, y._version, rmax, cmax))
    del _OPERAND_AMAX[:-4]


def _take_amax(x, rows, cols):
    """(row maxima, column maxima) of the [rows][cols] operand x if its producer left them."""
    for i, (y, ptr, r, c, ver, rmax, cmax) in enumerate(_OPERAND_AMAX):
        if ptr == x.data_ptr() and (r, c) == (rows, cols) and x.numel() == rows * cols \
                and x._version == ver == y._version and x.is_contiguous():
            del _OPERAND_AMAX[i]
            return rmax, cmax
    return None, None


def bn_apply_amax(x, rows, c, mean, invstd, gamma, beta):
    """bn_apply over [rows][c] that also keeps y's row / column maxima for the fp16x3 GEMMs
    reading it next (ds2_bn_apply_amax); plain bn_apply where its shape conditions fail."""
    ptrs = (x.data_ptr(), mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr())
    if c % 4 or c > 2048 or rows <= 0 or any(p % 16 for p in ptrs):
        return bn_apply(x, rows, c, 1, mean, invstd, gamma, beta)
    y = torch.empty_like(x)
    rmax = torch.empty(rows, dtype=_I32, device=x.device)
    cmax = torch.empty(c, dtype=_I32, device=x.device)
    _lib.call("ds2_bn_apply_amax", x.data_ptr(), rows, c, mean.data_ptr(), invstd.data_ptr(),
              gamma.data_ptr(), beta.data_ptr(), y.data_ptr(), rmax.data_ptr(), cmax.data_ptr(),
              _stream())
    _tag_amax(y, rows, c, rmax, cmax)
    return y


def bn_backward(dy, dy_layout, x, outer, c, d, t, mean, invstd, gamma, beta, masked=False,
                lens=None, lo=0.0, hi=20.0, want_dbias=False, bias=None):
    """dgamma / dbeta (/ dbias of the preceding conv) land in the parameters' gradient
    slots when they have one (grad_like)."""
    dx = torch.empty(outer, c, d, t, device=x.device, dtype=_F32)
    dgamma = grad_like(gamma)
    dbeta = grad_like(beta)
    dbias = None
    if want_dbias:
        dbias = grad_like(bias) if bias is not None else torch.empty(c, device=x.device,
                                                                      dtype=_F32)
    ws = _ws(_lib.size("ds2_bn_workspace_size", outer, c, d * t), x.device)
    _lib.call("ds2_bn_backward", dy.data_ptr(), dy_layout, x.data_ptr(), outer, c, d, t,
              mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(), int(masked),
              _p(lens), float(lo), float(hi), dx.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(),
              _p(dbias), ws.data_ptr(), ws.numel(), _stream())
    return dx, dgamma, dbeta, dbias


def colsum(x2d_storage, rows, cols, ld, out, accumulate=False, off=0):
    ws = _ws(_lib.size("ds2_colsum_workspace_size", rows, cols), out.device)
    _lib.call("ds2_colsum", x2d_storage.data_ptr() + 4 * off, rows, cols, ld, out.data_ptr(),
              int(accumulate), ws.data_ptr(), ws.numel(), _stream())
    return out


def softmax_tnc(logits_tnc: torch.Tensor) -> torch.Tensor:
    """probs[N,T,C] = softmax over C of logits stored [T,N,C]."""
    x = _need(logits_tnc, "softmax.logits")
    t, n, c = x.shape
    probs = torch.empty(n, t, c, device=x.device, dtype=_F32)
    _lib.call("ds2_softmax_tnc", x.data_ptr(), t, n, c, probs.data_ptr(), _stream())
    return probs


def ctc_loss_raw(acts_tnc, labels, act_lens, label_lens, max_label_len, blank=0,
                 zero_infinity=False, want_grad=True):
    acts = _need(acts_tnc, "ctc.acts")
    t, n, c = acts.shape
    costs = torch.empty(n, device=acts.device, dtype=_F32)
    grads = torch.empty_like(acts) if want_grad else None
    ws = _ws(_lib.size("ds2_ctc_workspace_size", t, n, max_label_len), acts.device)
    _lib.call("ds2_ctc_loss", acts.data_ptr(), t, n, c, labels.data_ptr(), label_lens.data_ptr(),
              act_lens.data_ptr(), int(max_label_len), int(blank), int(zero_infinity),
              costs.data_ptr(), _p(grads), ws.data_ptr(), ws.numel(), _stream())
    return costs, grads


def greedy_decode_raw(probs: torch.Tensor, sizes: Optional[torch.Tensor], blank: int = 0,
                      want_argmax: bool = False):
    """Device argmax + CTC collapse.  probs [N,T,C] (any strides, fp32).

    Returns (ids [N,T] int32, offsets [N,T] int32, counts [N] int32, argmax or None);
    row n holds counts[n] valid entries.
    """
    if not probs.is_cuda or probs.dtype != _F32:
        raise _lib.Ds2Error("greedy_decode: expected a float32 device tensor")
    n, t, c = probs.shape
    if probs.stride(2) != 1:
        probs = probs.contiguous()
    ids = torch.empty(n, t, device=probs.device, dtype=_I32)
    offs = torch.empty(n, t, device=probs.device, dtype=_I32)
    counts = torch.empty(n, device=probs.device, dtype=_I32)
    am = torch.empty(n, t, device=probs.device, dtype=_I32) if want_argmax else None
    if sizes is not None:
        sizes = sizes.to(device=probs.device, dtype=_I32).contiguous()
    _lib.call("ds2_greedy_decode", probs.data_ptr(), n, t, c, probs.stride(0), probs.stride(1),
              _p(sizes), int(blank), ids.data_ptr(), offs.data_ptr(), counts.data_ptr(), _p(am),
              _stream())
    return ids, offs, counts, am


def edit_distance_raw(a_ids: torch.Tensor, a_lens: torch.Tensor, b_ids: torch.Tensor,
                      b_lens: torch.Tensor, space_id: int):
    """Device CER/WER distances.  a_ids [N, S] int32 rows with a_lens valid; b_ids flat int32
    (concatenated references), b_lens [N].  Returns int32 [N, 4] = (word dist, char dist,
    max(#ref words, 1), max(#ref chars, 1)); raises if a sequence exceeds the kernel limits."""
    dev = a_ids.device
    if not a_ids.is_cuda:
        raise _lib.Ds2Error("edit_distance: expected device tensors")
    a_ids = a_ids.to(_I32).contiguous()
    a_lens = a_lens.to(device=dev, dtype=_I32).contiguous()
    b_ids = b_ids.to(device=dev, dtype=_I32).contiguous()
    b_lens = b_lens.to(device=dev, dtype=_I32).contiguous()
    b_off = (torch.cumsum(b_lens, 0) - b_lens).to(_I32).contiguous()
    n = a_ids.shape[0]
    out = torch.empty(n, 4, device=dev, dtype=_I32)
    err = torch.zeros(1, device=dev, dtype=_I32)
    _lib.call("ds2_edit_distance", a_ids.data_ptr(), a_ids.stride(0), a_lens.data_ptr(),
              b_ids.data_ptr(), b_off.data_ptr(), b_lens.data_ptr(), n, int(space_id),
              out.data_ptr(), err.data_ptr(), _stream())
    return out, err


def ctc_beam_decode_raw(probs: torch.Tensor, sizes: Optional[torch.Tensor], beam_width: int,
                        top_paths: int, blank: int = 0, cutoff_top_n: int = 40,
                        cutoff_prob: float = 1.0):
    """Device CTC prefix beam search (no LM).  probs [N,T,C] fp32 (any strides).

    Returns (ids [N,P,T] int32, offsets [N,P,T] int32, lens [N,P] int32, scores [N,P]
    fp32), paths best first; row (n, p) holds lens[n, p] valid entries.
    """
    if not probs.is_cuda or probs.dtype != _F32:
        raise _lib.Ds2Error("ctc_beam_decode: expected a float32 device tensor")
    n, t, c = probs.shape
    if probs.stride(2) != 1:
        probs = probs.contiguous()
    dev = probs.device
    ids = torch.empty(n, top_paths, t, device=dev, dtype=_I32)
    offs = torch.empty(n, top_paths, t, device=dev, dtype=_I32)
    lens = torch.empty(n, top_paths, device=dev, dtype=_I32)
    scores = torch.empty(n, top_paths, device=dev, dtype=_F32)
    if sizes is not None:
        sizes = sizes.to(device=dev, dtype=_I32).contiguous()
    ws = _ws(_lib.size("ds2_ctc_beam_workspace_size", n, t, beam_width), dev)
    _lib.call("ds2_ctc_beam_decode", probs.data_ptr(), n, t, c, probs.stride(0), probs.stride(1),
              _p(sizes), int(blank), int(beam_width), int(cutoff_top_n), float(cutoff_prob),
              int(top_paths), ids.data_ptr(), offs.data_ptr(), lens.data_ptr(), scores.data_ptr(),
              ws.data_ptr(), ws.numel(), _stream())
    return ids, offs, lens, scores


def ctc_beam_decode_lm_raw(probs: torch.Tensor, sizes: Optional[torch.Tensor], beam_width: int,
                           top_paths: int, scorer, blank: int = 0, cutoff_top_n: int = 40,
                           cutoff_prob: float = 1.0):
    """ctc_beam_decode_raw with a word n-gram LM (scorer: ds2amd.lm.ArpaScorer, its tables
    on the same device).  Same outputs; scores include the LM terms."""
    if not probs.is_cuda or probs.dtype != _F32:
        raise _lib.Ds2Error("ctc_beam_decode_lm: expected a float32 device tensor")
    n, t, c = probs.shape
    if probs.stride(2) != 1:
        probs = probs.contiguous()
    dev = probs.device
    if scorer.table.device != dev:
        raise _lib.Ds2Error("ctc_beam_decode_lm: the LM tables live on another device")
    if scorer.dict_next.shape[1] != c:
        raise _lib.Ds2Error("ctc_beam_decode_lm: the LM was built for another label set")
    ids = torch.empty(n, top_paths, t, device=dev, dtype=_I32)
    offs = torch.empty(n, top_paths, t, device=dev, dtype=_I32)
    lens = torch.empty(n, top_paths, device=dev, dtype=_I32)
    scores = torch.empty(n, top_paths, device=dev, dtype=_F32)
    if sizes is not None:
        sizes = sizes.to(device=dev, dtype=_I32).contiguous()
    ws = _ws(_lib.size("ds2_ctc_beam_workspace_size", n, t, beam_width), dev)
    _lib.call("ds2_ctc_beam_decode_lm", probs.data_ptr(), n, t, c, probs.stride(0),
              probs.stride(1), _p(sizes), int(blank), int(beam_width), int(cutoff_top_n),
              float(cutoff_prob), int(top_paths), scorer.space, scorer.order, scorer.start_id,
              len(scorer.vocab), scorer.alpha, scorer.beta, scorer.dict_next.data_ptr(),
              scorer.dict_mask.data_ptr(), scorer.dict_word.data_ptr(), scorer.n_states,
              int(scorer.dict_next.shape[1]), scorer.table.data_ptr(),
              scorer.table_mask + 1, ids.data_ptr(), offs.data_ptr(), lens.data_ptr(),
              scores.data_ptr(), ws.data_ptr(), ws.numel(), _stream())
    return ids, offs, lens, scores


def wave_aug(pcm: torch.Tensor, in_lens: torch.Tensor, op_i: torch.Tensor, op_f: torch.Tensor,
             noise: Optional[torch.Tensor], out_lens, out_stride: int, cap: int,
             check: bool = True) -> torch.Tensor:
    """Replay host-drawn waveform-augmentation records on the device (ds2_wave_aug).
    pcm [N, S] fp32, in_lens int32 [N], op_i int32 [N, K, 4], op_f float64 [N, K],
    noise float64 [R, L] or None -> [N, out_stride] fp32 zero padded.  check=False skips the
    blocking read of the kernel's consistency word, for callers that validated the records
    on the host (audio_aug.apply_waves)."""
    pcm = _need(pcm, "wave_aug.pcm")
    in_lens = _need(in_lens, "wave_aug.in_lens", _I32)
    op_i = _need(op_i, "wave_aug.op_i", _I32)
    op_f = _need(op_f, "wave_aug.op_f", torch.float64)
    n, k = op_i.shape[0], op_i.shape[1]
    dev = pcm.device
    if noise is not None:
        noise = _need(noise, "wave_aug.noise", torch.float64)
    out_lens = _need(torch.as_tensor(out_lens, dtype=_I32).to(dev), "wave_aug.out_lens", _I32)
    out = torch.empty(n, out_stride, device=dev, dtype=_F32)
    err = torch.zeros(1, device=dev, dtype=_I32)
    ws = _ws(_lib.size("ds2_wave_aug_workspace_size", n, cap), dev)
    _lib.call("ds2_wave_aug", pcm.data_ptr(), pcm.stride(0), in_lens.data_ptr(), n, op_i.data_ptr(),
              op_f.data_ptr(), k, _p(noise), 0 if noise is None else noise.stride(0),
              out.data_ptr(), out_stride, out_lens.data_ptr(), cap, err.data_ptr(), ws.data_ptr(),
              ws.numel(), _stream())
    if check and int(err.item()) != 0:
        raise _lib.Ds2Error(f"ds2_wave_aug: inconsistent op records (err {int(err.item())})")
    return out


# librosa / resampy effects (csrc/effects.hip): ChangeAudioSpeed, PitchShift, resampling
FX_N_FFT, FX_HOP = 2048, 512


def hann_periodic(n: int) -> np.ndarray:
    """scipy.signal.get_window('hann', n, fftbins=True): general_cosine over n + 1 points,
    last one dropped (same float64 operations as scipy)."""
    fac = np.linspace(-np.pi, np.pi, n + 1)
    w = np.zeros(n + 1)
    w += 0.5 * np.cos(0 * fac)
    w += 0.5 * np.cos(fac)
    return w[:-1]


_FX_CONST = {}


def _fx_window(dev):
    key = ('hann', dev)
    if key not in _FX_CONST:
        _FX_CONST[key] = torch.from_numpy(hann_periodic(FX_N_FFT)).to(dev)
    return _FX_CONST[key]


def kaiser_best_filter() -> tuple:
    """resampy 'kaiser_best': sinc_window(num_zeros=64, precision=9,
    window=kaiser(beta=14.769656459379492), rolloff=0.9475937167399596) -> (right wing
    float64 [64 * 512 + 1], 512 samples per zero crossing)."""
    from scipy.signal.windows import kaiser
    num_zeros, num_bits, beta, rolloff = 64, 2 ** 9, 14.769656459379492, 0.9475937167399596
    n = num_bits * num_zeros
    sinc_win = rolloff * np.sinc(rolloff * np.linspace(0, num_zeros, num=n + 1, endpoint=True))
    taper = kaiser(2 * n + 1, beta)[n:]
    return taper * sinc_win, num_bits


def _fx_filter(dev):
    key = ('kaiser_best', dev)
    if key not in _FX_CONST:
        win, nb = kaiser_best_filter()
        _FX_CONST[key] = (torch.from_numpy(np.ascontiguousarray(win)).to(dev), nb)
    return _FX_CONST[key]


def stretch_plan(in_len: int, rate: float) -> tuple:
    """(out_len, out_frames, used_frames) of librosa.effects.time_stretch(y, rate) for a
    len-in_len y: round(len / rate) (Python round), ceil(frames / rate) (np.arange length),
    min(that, ceil((out_len + n_fft) / hop)) (istft's length-limited frame count)."""
    import math
    frames = 1 + in_len // FX_HOP
    out_len = int(round(in_len / rate))
    out_frames = int(math.ceil((frames - 0) / rate))
    used = min(out_frames, int(math.ceil((out_len + FX_N_FFT) / FX_HOP)))
    return out_len, out_frames, used


def time_stretch(pcm: torch.Tensor, lens, rates) -> tuple:
    """Per-utterance librosa.effects.time_stretch on the device (ds2_time_stretch).
    pcm [N, S] fp32 device, lens / rates host sequences -> (out [N, max out_len], out_lens)."""
    pcm = _need(pcm, "time_stretch.pcm")
    n = pcm.shape[0]
    dev = pcm.device
    plans = [stretch_plan(int(l), float(r)) for l, r in zip(lens, rates)]
    out_lens = [p[0] for p in plans]
    stride = max(1, max(out_lens) if out_lens else 1)
    max_in = max([1 + int(l) // FX_HOP for l in lens] or [1])
    max_out = max([p[1] for p in plans] or [1])
    i32 = lambda v: torch.tensor(v, dtype=_I32).to(dev)
    out = torch.empty(n, stride, device=dev, dtype=_F32)
    ws = _ws(_lib.size("ds2_time_stretch_workspace_size", n, max_in, max_out), dev)
    lens_d, rate_d = i32([int(l) for l in lens]), torch.tensor([float(r) for r in rates],
                                                               dtype=torch.float64).to(dev)
    of_d, uf_d, ol_d = i32([p[1] for p in plans]), i32([p[2] for p in plans]), i32(out_lens)
    _lib.call("ds2_time_stretch", pcm.data_ptr(), pcm.stride(0), lens_d.data_ptr(), n,
              rate_d.data_ptr(), of_d.data_ptr(), uf_d.data_ptr(), ol_d.data_ptr(),
              _fx_window(dev).data_ptr(), out.data_ptr(), stride, max_in, max_out, ws.data_ptr(),
              ws.numel(), _stream())
    return out, out_lens


def resample(pcm: torch.Tensor, lens, ratios, out_lens=None) -> tuple:
    """Per-utterance resampy 'kaiser_best' resampling on the device (ds2_resample).
    ratios = sr_new / sr_orig (float64 as numpy forms it); each utterance yields
    int(len * ratio) samples, zero-padded to out_lens (default: that count)."""
    pcm = _need(pcm, "resample.pcm")
    n = pcm.shape[0]
    dev = pcm.device
    valid = [int(int(l) * float(r)) for l, r in zip(lens, ratios)]
    if out_lens is None:
        out_lens = valid
    stride = max(1, max(out_lens) if len(out_lens) else 1)
    out = torch.empty(n, stride, device=dev, dtype=_F32)
    win, nb = _fx_filter(dev)
    ws = _ws(_lib.size("ds2_resample_workspace_size", n, stride), dev)
    lens_d = torch.tensor([int(l) for l in lens], dtype=_I32).to(dev)
    valid_d = torch.tensor([min(v, o) for v, o in zip(valid, out_lens)], dtype=_I32).to(dev)
    ratio_d = torch.tensor([float(r) for r in ratios], dtype=torch.float64).to(dev)
    _lib.call("ds2_resample", pcm.data_ptr(), pcm.stride(0), lens_d.data_ptr(), n,
              ratio_d.data_ptr(), valid_d.data_ptr(), win.data_ptr(), win.numel(), nb,
              out.data_ptr(), stride, ws.data_ptr(), ws.numel(), _stream())
    return out, list(out_lens)


SPECT_ROWS = 161   # rows of every spectrogram the reference returns (data_loader_aug.py:234-249)


def stft_logmag(pcm: torch.Tensor, n_samples: torch.Tensor, n_fft: int, hop: int,
                window: torch.Tensor, normalize: int, gauss_taps: Optional[torch.Tensor],
                max_frames: int, masks: Optional[torch.Tensor] = None) -> torch.Tensor:
    """-> [batch, 161, max_frames]: the first 161 bins, or the reference's mirror-fill when
    n_fft/2+1 < 161 (8 kHz audio; ds2hip.h).  masks: None or int32 [batch, 9]
    spectrogram-augmentation bands (ds2hip.h), rows of the 161-row output."""
    pcm = _need(pcm, "stft.pcm")
    n_samples = _need(n_samples, "stft.n_samples", _I32)
    window = _need(window, "stft.window", torch.float64)
    b, max_samples = pcm.shape
    out = torch.empty(b, SPECT_ROWS, max_frames, device=pcm.device, dtype=_F32)
    ws = _ws(_lib.size("ds2_stft_workspace_size", b, max_frames, n_fft), pcm.device)
    radius = 0 if gauss_taps is None else (gauss_taps.numel() - 1) // 2
    if masks is not None:
        masks = _need(masks, "stft.masks", _I32)
        if tuple(masks.shape) != (b, 9):
            raise _lib.Ds2Error(f"stft masks must be [batch, 9], got {tuple(masks.shape)}")
    _lib.call("ds2_stft_logmag_masked", pcm.data_ptr(), n_samples.data_ptr(), b, max_samples,
              n_fft, hop, window.data_ptr(), int(normalize), _p(gauss_taps), radius, _p(masks),
              out.data_ptr(), max_frames, ws.data_ptr(), ws.numel(), _stream())
    return out


# ----------------------------------------------------------------------------
# autograd functions
class ConvBlockFn(torch.autograd.Function):
    """Conv2d -> mask -> BatchNorm2d -> mask -> Hardtanh -> mask (model.py:208-215,63-79).

    out_layout 0 returns [N, C, D, T'] like MaskConv; 1 returns the T'xNx(C*D)
    collapse of model.py:360-362 directly.
    """

    @staticmethod
    def forward(ctx, x, lens, weight, bias, gamma, beta, running_mean, running_var, training,
                momentum, eps, stride, padding, lo, hi, out_layout):
        z = conv2d_fwd(x, weight, bias, stride, padding, out_lens=lens)
        n, c, d, t = z.shape
        mean, invstd = bn_stats(z, n, c, d * t, eps, momentum, running_mean, running_var, training)
        if out_layout == 1:
            y = torch.empty(t, n, c * d, device=z.device, dtype=_F32)
        else:
            y = torch.empty_like(z)
        _lib.call("ds2_bn_apply_mask_htanh", z.data_ptr(), n, c, d, t, mean.data_ptr(),
                  invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(), _p(lens), float(lo),
                  float(hi), y.data_ptr(), int(out_layout), _stream())
        ctx.save_for_backward(x, z, lens, weight, gamma, beta, mean, invstd)
        ctx.bias = bias   # only its identity (gradient slot) is used in backward
        ctx.cfg = (stride, padding, lo, hi, out_layout, bias is not None, training)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, z, lens, weight, gamma, beta, mean, invstd = ctx.saved_tensors
        stride, padding, lo, hi, out_layout, has_bias, training = ctx.cfg
        if not training:
            raise _lib.Ds2Error("ConvBlockFn backward in eval mode is not supported")
        dy = dy.contiguous()
        n, c, d, t = z.shape
        dz, dgamma, dbeta, dbias = bn_backward(dy, out_layout, z, n, c, d, t, mean, invstd, gamma,
                                               beta, masked=True, lens=lens, lo=lo, hi=hi,
                                               want_dbias=has_bias, bias=ctx.bias)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = conv2d_dgrad(dz, weight, x.shape, stride, padding)
        dw, _ = conv2d_wgrad(dz, x, weight.shape, stride, padding, with_bias=False,
                             out_dw=grad_like(weight))
        return (dx, None, dw, dbias, dgamma, dbeta) + (None,) * 10


class SeqBatchNormFn(torch.autograd.Function):
    """SequenceWise(BatchNorm1d) on x viewed [R, C] (model.py:28-43, 89, 336)."""

    @staticmethod
    def forward(ctx, x2d, gamma, beta, running_mean, running_var, training, momentum, eps):
        x2d = x2d.contiguous()
        r, c = x2d.shape
        mean, invstd = bn_stats(x2d, r, c, 1, eps, momentum, running_mean, running_var, training)
        # with the fp16x3 GEMMs, y's row / column maxima for the input projection and dW_ih
        y = (bn_apply_amax(x2d, r, c, mean, invstd, gamma, beta) if h3_enabled()
             else bn_apply(x2d, r, c, 1, mean, invstd, gamma, beta))
        ctx.save_for_backward(x2d, gamma, beta, mean, invstd)
        ctx.training = training
        return y

    @staticmethod
    def backward(ctx, dy):
        x2d, gamma, beta, mean, invstd = ctx.saved_tensors
        if not ctx.training:
            raise _lib.Ds2Error("SeqBatchNormFn backward in eval mode is not supported")
        r, c = x2d.shape
        dx, dgamma, dbeta, _ = bn_backward(dy.contiguous(), 0, x2d, r, c, 1, 1, mean, invstd,
                                           gamma, beta)
        return dx.view(r, c), dgamma, dbeta, None, None, None, None, None


class LinearFn(torch.autograd.Function):
    """y = x @ W^T (no bias; model.py:337)."""

    @staticmethod
    def forward(ctx, x2d, weight):
        x2d = x2d.contiguous()
        ctx.save_for_backward(x2d, weight)
        # the fp16x3 scales of x the BatchNorm before it kept (the FC's SequenceWise BN): rows
        # for this GEMM, columns for dW's
        m, k = x2d.shape
        x_r, ctx.x_c = _take_amax(x2d, m, k) if h3_enabled() else (None, None)
        out = torch.empty(m, weight.shape[0], device=x2d.device, dtype=_F32)
        return sgemm(x2d, weight, out, m=m, n=weight.shape[0], k=k, trans_b=True, lda=k, ldb=k,
                     ldc=weight.shape[0], a_amax=x_r)

    @staticmethod
    def backward(ctx, dy):
        x2d, weight = ctx.saved_tensors
        dy = dy.contiguous()
        m, k = x2d.shape
        n = weight.shape[0]
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x2d)
            sgemm(dy, weight, dx, m=m, n=k, k=n, lda=n, ldb=k, ldc=k)
        dw = grad_like(weight)
        sgemm(dy, x2d, dw, m=n, n=k, k=m, trans_a=True, lda=n, ldb=k, ldc=k, b_amax=ctx.x_c)
        return dx, dw


# Precision of the recurrent layers' GEMMs (input projection, dX, dW_ih, dW_hh): fp32 by
# default (parity with the reference's fp32 path); bf16 operands on the bf16 MFMA with fp32
# accumulation as BASELINE cfg4's opt-in ("bf16 MFMA RNN GEMMs").  Set around one layer
# call by rnn_gemm_precision(); the autograd Functions record it for their backward.
_RNN_GEMM_BF16 = [False]


class rnn_gemm_precision:
    """Context manager: ``with rnn_gemm_precision('bf16'): y = GRULayerFn.apply(...)``."""

    def __init__(self, precision: str):
        if precision not in ('fp32', 'bf16'):
            raise ValueError(f"rnn GEMM precision must be 'fp32' or 'bf16', got {precision!r}")
        self.bf16 = precision == 'bf16'

    def __enter__(self):
        self.prev = _RNN_GEMM_BF16[0]
        _RNN_GEMM_BF16[0] = self.bf16
        return self

    def __exit__(self, *exc):
        _RNN_GEMM_BF16[0] = self.prev
        return False


def _stacked_rows(a: torch.Tensor, b: torch.Tensor):
    """[a; b] as one row-major matrix when b starts where a ends in the same storage (the
    layout optim.FlatParams gives a bidirectional layer's W_ih pair and its gradient
    slots), else None."""
    if a.dim() != 2 or tuple(b.shape) != tuple(a.shape) or not (a.is_contiguous() and
                                                                   b.is_contiguous()):
        return None
    if a.untyped_storage().data_ptr() != b.untyped_storage().data_ptr():
        return None
    if b.data_ptr() != a.data_ptr() + a.numel() * a.element_size():
        return None
    return a.as_strided((2 * a.shape[0], a.shape[1]), (a.shape[1], 1))


def _rnn_input_proj(x, weights, nd, g, bf16=False, need_dx=False):
    """(xproj, pre): xproj[T, N, D, g] = x @ W_ih^T + b_ih for every direction, one GEMM over
    both directions when their W_ih lie back to back (N = 2g), else one GEMM each.  With the
    fp16x3 GEMMs, x's row maxima come from the kernel that produced x where it kept them
    (ds2_bn_apply_amax) and the stacked W_ih's row maxima from one pass that also takes its
    column maxima when the backward's dX GEMM will need them; ``pre`` hands the column maxima
    of x and W_ih to _rnn_param_grads, which would otherwise re-read both operands."""
    t, n, inp = x.shape
    x2d = x.view(t * n, inp)
    xproj = torch.empty(t, n, nd, g, device=x.device, dtype=_F32)
    ws = _stacked_rows(weights[0], weights[4]) if nd == 2 else None
    pre = {}
    x_r = w_r = None
    if h3_enabled() and not bf16:
        x_r, pre["x_c"] = _take_amax(x2d, t * n, inp)
        if pre["x_c"] is None:
            del pre["x_c"]
        elif ws is not None:
            w_r, w_c = amax(ws, 2 * g, inp, inp, want_cols=need_dx)
            if w_c is not None:
                pre["w_c"] = w_c
    if ws is not None:
        bias = torch.cat([weights[2], weights[6]])
        sgemm(x2d, ws, xproj, m=t * n, n=2 * g, k=inp, trans_b=True, lda=inp, ldb=inp,
              ldc=2 * g, bias=bias, bf16=bf16, a_amax=x_r, b_amax=w_r)
        return xproj, pre
    for d in range(nd):
        w_ih, _, b_ih, _ = weights[4 * d: 4 * d + 4]
        sgemm(x2d, w_ih, xproj, m=t * n, n=g, k=inp, trans_b=True, lda=inp, ldb=inp,
              ldc=nd * g, bias=b_ih, c_off=d * g, bf16=bf16, a_amax=x_r)
    return xproj, pre


def _rnn_output(h_all, sum_dirs, nd):
    t, n, _, h = h_all.shape
    if sum_dirs and nd == 2:
        y = torch.empty(t, n, h, device=h_all.device, dtype=_F32)
        _lib.call("ds2_dirsum", h_all.data_ptr(), t * n, nd, h, y.data_ptr(), _stream())
        return y
    return h_all.view(t, n, nd * h)


def _rnn_param_grads_bf16(x2d, h_all, dgx, dgh, weights, nd, g, t, n, inp, h, need_dx, dbias):
    """_rnn_param_grads with bf16 operands (BASELINE cfg4's opt-in) on ds2_bgemm_nt, each
    operand rounded to bf16 ONCE per layer into the k-contiguous copy the GEMMs share:
    dgx^T [D g][T N] serves dW_ih (all rows) and, shifted by one step, dW_hh (the LSTM's dgh is
    dgx); x^T and h^T likewise; dgx as is serves dX.  Same rounding (RNE) and products as the
    per-GEMM conversions of sgemm(..., bf16=True); only where the copies come from differs."""
    dev = x2d.device
    tn = t * n
    ld = nd * g
    dgx2 = dgx.view(tn, ld)
    dgx_t = to_bf16(dgx2, transpose=True)                       # [ld][tn]
    dgh_t = dgx_t if dgh is dgx else to_bf16(dgh.view(tn, ld), transpose=True)
    x_t = to_bf16(x2d, transpose=True)                          # [inp][tn]
    h_t = to_bf16(h_all.view(tn, nd * h), transpose=True)       # [nd h][tn]
    dx = torch.empty(t, n, inp, device=dev, dtype=_F32) if need_dx else None
    grads = []
    if dx is not None:
        dgx_b = to_bf16(dgx2)                                   # [tn][ld]
        w_all = torch.cat([weights[4 * d] for d in range(nd)], 0) if nd > 1 else weights[0]
        w_t = to_bf16(w_all, transpose=True)                    # [inp][ld]
        bgemm_nt(dgx_b, w_t, dx.view(tn, inp))
    for d in range(nd):
        w_ih, w_hh, b_ih, b_hh = weights[4 * d: 4 * d + 4]
        dw_ih = grad_like(w_ih)
        bgemm_nt(dgx_t[d * g:(d + 1) * g], x_t, dw_ih)
        if dbias is not None:
            db_ih, db_hh = dbias[2 * d], dbias[2 * d + 1]
        else:
            db_ih = grad_like(b_ih)
            colsum(dgx, tn, g, ld, db_ih, off=d * g)
        # sum_t dgh_t^T h_{t-1} (fwd) / h_{t+1} (rev): k runs over (t - 1) n rows, dgh from
        # step 1 (fwd) or 0 (rev), h from step 0 (fwd) or 1 (rev)
        k = (t - 1) * n
        ka, kb = (n, 0) if d == 0 else (0, n)
        dw_hh = grad_like(w_hh)
        bgemm_nt(dgh_t[d * g:(d + 1) * g, ka:ka + k], h_t[d * h:(d + 1) * h, kb:kb + k], dw_hh)
        if dbias is None:
            db_hh = grad_like(b_hh)
            if dgh is dgx:
                db_hh.copy_(db_ih)
            elif g == 3 * h:
                db_hh[:2 * h].copy_(db_ih[:2 * h])
                colsum(dgh, tn, h, ld, db_hh[2 * h:], off=d * g + 2 * h)
            else:
                colsum(dgh, tn, g, ld, db_hh, off=d * g)
        grads += [dw_ih, dw_hh, db_ih, db_hh]
    return dx, grads


def _rnn_param_grads(x, h_all, dgx, dgh, weights, nd, g, need_dx, bf16=False, pre=None,
                     dbias=None, shared_bf16=True, col_amax=None):
    """Weight/bias/input gradients of one recurrent layer from the gate gradients.

    dgx = d/d(x W_ih^T + b_ih), dgh = d/d(h W_hh^T + b_hh), both [T, N, D, g]
    (the same tensor for LSTM).  All plain GEMMs + column sums; dbias = [db_ih, db_hh] per
    direction already summed (the GRU backward kernel's own sums) skips the column sums.
    shared_bf16=False keeps bf16 mode on the per-GEMM conversions (the cross-check of
    _rnn_param_grads_bf16's shared copies, tests/test_gpu_ops.py).  col_amax: the column
    maxima of dgx and dgh ([2 D g] float bits) when the recurrence kept them.  pre: the column
    maxima of x and of the stacked W_ih the forward's input projection took (_rnn_input_proj).
    """
    t, n, inp = x.shape
    h = h_all.shape[-1]
    dev = x.device
    x2d = x.view(t * n, inp)
    tn = t * n
    ld = nd * g
    if bf16 and shared_bf16 and t > 1 and all(v % 8 == 0 for v in (n, inp, h, g)):
        return _rnn_param_grads_bf16(x2d, h_all, dgx, dgh, weights, nd, g, t, n, inp, h,
                                     need_dx, dbias)
    grads = []
    dx = torch.empty(t, n, inp, device=dev, dtype=_F32) if need_dx else None
    # both directions in one GEMM where W_ih (dX) and its gradient slots (dW_ih) are stacked
    w_st = _stacked_rows(weights[0], weights[4]) if nd == 2 else None
    dw_ih_all = [grad_like(weights[4 * d]) for d in range(nd)]
    dw_st = _stacked_rows(dw_ih_all[0], dw_ih_all[1]) if w_st is not None else None
    # fp16x3 operand scales, each operand read once and shared by the GEMMs below: dgx rows
    # (dX) and columns (dW_ih), dgh columns (dW_hh; a bound over all its rows), x and W_ih
    # columns, and 1.0 for the tanh-bounded states h
    am = {}
    if h3_enabled() and not bf16:
        if col_amax is not None:
            # [2 D g] (dgx, dgh), or [D g] when dgh is dgx (the one-gate RNN)
            am["dgx_c"] = col_amax[:ld]
            am["dgh_c"] = col_amax[ld:] if col_amax.numel() == 2 * ld else am["dgx_c"]
            if need_dx:
                am["dgx_r"] = amax(dgx, tn, ld, ld, want_cols=False)[0]
        else:
            am["dgx_r"], am["dgx_c"] = amax(dgx, tn, ld, ld, want_rows=need_dx)
            am["dgh_c"] = am["dgx_c"] if dgh is dgx else amax(dgh, tn, ld, ld, want_rows=False)[1]
        pre = pre or {}
        am["x_c"] = pre["x_c"] if "x_c" in pre else amax(x2d, tn, inp, inp, want_rows=False)[1]
        am["h"] = unit_bound(nd * h, dev)
        if need_dx:
            if w_st is not None:
                am["w_c"] = (pre["w_c"] if "w_c" in pre
                             else amax(w_st, 2 * g, inp, inp, want_rows=False)[1])
            else:
                am["w_c"] = [amax(weights[4 * d], g, inp, inp, want_rows=False)[1]
                             for d in range(nd)]

    def sl(key, lo, hi):
        v = am.get(key)
        return None if v is None else v[lo:hi]

    if dw_st is not None:
        sgemm(dgx, x2d, dw_st, m=2 * g, n=inp, k=tn, trans_a=True, lda=ld, ldb=inp, ldc=inp,
              bf16=bf16, a_amax=am.get("dgx_c"), b_amax=am.get("x_c"))
    if dx is not None and w_st is not None:
        sgemm(dgx, w_st, dx, m=tn, n=inp, k=2 * g, lda=ld, ldb=inp, ldc=inp, bf16=bf16,
              a_amax=am.get("dgx_r"), b_amax=am.get("w_c"))
    for d in range(nd):
        w_ih, w_hh, b_ih, b_hh = weights[4 * d: 4 * d + 4]
        dw_ih = dw_ih_all[d]
        if dw_st is None:
            sgemm(dgx, x2d, dw_ih, m=g, n=inp, k=tn, trans_a=True, lda=ld, ldb=inp, ldc=inp,
                  a_off=d * g, bf16=bf16, a_amax=sl("dgx_c", d * g, (d + 1) * g),
                  b_amax=am.get("x_c"))
        if dbias is not None:
            db_ih, db_hh = dbias[2 * d], dbias[2 * d + 1]
        else:
            db_ih = grad_like(b_ih)
            colsum(dgx, tn, g, ld, db_ih, off=d * g)
        dw_hh = grad_like(w_hh)
        if t > 1:
            # sum_t dgh_t^T h_{t-1} (fwd) / h_{t+1} (rev); h_prev = 0 at the start
            a_off = (n * ld if d == 0 else 0) + d * g
            b_off = (0 if d == 0 else n * nd * h) + d * h
            sgemm(dgh, h_all, dw_hh, m=g, n=h, k=(t - 1) * n, trans_a=True, lda=ld,
                  ldb=nd * h, ldc=h, a_off=a_off, b_off=b_off, bf16=bf16,
                  a_amax=sl("dgh_c", d * g, (d + 1) * g), b_amax=sl("h", d * h, (d + 1) * h))
        else:
            dw_hh.zero_()
        if dbias is None:
            db_hh = grad_like(b_hh)
            if dgh is dgx:
                db_hh.copy_(db_ih)
            elif g == 3 * h:
                # GRU: the r and z columns of dgh are dgx's (the kernels store the same
                # values), so only the n third needs its own column sum
                db_hh[:2 * h].copy_(db_ih[:2 * h])
                colsum(dgh, tn, h, ld, db_hh[2 * h:], off=d * g + 2 * h)
            else:
                colsum(dgh, tn, g, ld, db_hh, off=d * g)
        if dx is not None and w_st is None:
            # dgx's row maxima span both directions: an upper bound for each direction's slice
            sgemm(dgx, w_ih, dx, m=tn, n=inp, k=g, lda=ld, ldb=inp, ldc=inp,
                  beta=0.0 if d == 0 else 1.0, a_off=d * g, bf16=bf16,
                  a_amax=am.get("dgx_r"), b_amax=None if "w_c" not in am else am["w_c"][d])
        grads += [dw_ih, dw_hh, db_ih, db_hh]
    return dx, grads


# Cooperative-launch guard (optim.GradAllReducer.guard_cooperative): called with the persistent
# recurrence's workgroup count before each backward launch, while gradient all-reduces of the
# same step may be in flight on RCCL's stream.
_COOP_GUARD = [None]


def set_cooperative_guard(fn) -> None:
    _COOP_GUARD[0] = fn


def persistent_bwd_grid(cell: str, n: int, h: int, nd: int) -> int:
    """Workgroups the persistent backward recurrence of this shape holds at once, as the
    library will launch it (ds2_gru_bwd_grid / ds2_lstm_bwd_grid / ds2_rnn_bwd_grid; 0 for the per-step
    kernels, which need no co-residency)."""
    fn = {"gru": "ds2_gru_bwd_grid", "lstm": "ds2_lstm_bwd_grid", "rnn": "ds2_rnn_bwd_grid",
          "lstm_half": "ds2_lstm_bwd_half_grid"}[cell]
    return _lib.size(fn, n, h, nd)


def _guard_cooperative(cell, n, h, nd):
    g = _COOP_GUARD[0]
    if g is not None:
        grid = persistent_bwd_grid(cell, n, h, nd)
        if grid > 0:
            g(grid)


class GRULayerFn(torch.autograd.Function):
    """One (bi)directional GRU layer over padded [T, N, In] input with lengths.

    Equals pack_padded_sequence -> nn.GRU -> pad_packed_sequence (model.py:103-105);
    with sum_dirs it also folds the direction sum of model.py:107.
    """

    @staticmethod
    def forward(ctx, x, lens, sum_dirs, hidden, *weights):
        x = x.contiguous()
        t, n, _ = x.shape
        h = hidden
        nd = len(weights) // 4
        dev = x.device
        bf16 = _RNN_GEMM_BF16[0]
        xproj, ctx.pre = _rnn_input_proj(x, weights, nd, 3 * h, bf16, ctx.needs_input_grad[0])
        h_all = torch.empty(t, n, nd, h, device=dev, dtype=_F32)
        need_grad = any(ctx.needs_input_grad)   # forward() itself runs under no_grad
        # backward cache: [T][N][D][4H] gates + the dh-exchange backward's coefficient tiles
        gates = (torch.empty(_lib.size("ds2_gru_cache_floats", t, n, h, nd), device=dev,
                             dtype=_F32) if need_grad else None)
        w_hh_f, b_hh_f = weights[1], weights[3]
        w_hh_r = weights[5] if nd == 2 else None
        b_hh_r = weights[7] if nd == 2 else None
        ws = _ws(_lib.size("ds2_gru_fwd_workspace_size", n, h, nd), dev)
        _lib.call("ds2_gru_fwd", t, n, h, nd, xproj.data_ptr(), w_hh_f.data_ptr(), _p(w_hh_r),
                  b_hh_f.data_ptr(), _p(b_hh_r), lens.data_ptr(), h_all.data_ptr(), _p(gates),
                  rnn_status_word(dev).data_ptr(), ws.data_ptr(), ws.numel(), _stream())
        ctx.save_for_backward(x, lens, h_all, gates, *weights)
        ctx.cfg = (sum_dirs, h, nd, bf16)
        return _rnn_output(h_all, sum_dirs, nd)

    @staticmethod
    def backward(ctx, dy):
        x, lens, h_all, gates, *weights = ctx.saved_tensors
        sum_dirs, h, nd, bf16 = ctx.cfg
        t, n, _ = x.shape
        dev = x.device
        h3 = 3 * h
        dy = dy.contiguous()
        dy_dirs = 1 if (sum_dirs and nd == 2) else nd
        dgx = torch.empty(t, n, nd, h3, device=dev, dtype=_F32)
        dgh = torch.empty(t, n, nd, h3, device=dev, dtype=_F32)
        w_hh_f = weights[1]
        w_hh_r = weights[5] if nd == 2 else None
        ws = _ws(_lib.size("ds2_gru_bwd_workspace_size", n, h, nd), dev)
        _guard_cooperative("gru", n, h, nd)
        # bias gradients straight into their slots, summed by the recurrence kernel; with the
        # fp16x3 GEMMs the kernel also keeps the column maxima of dgx / dgh they scale by
        dbias = [grad_like(weights[4 * d + k]) for d in range(nd) for k in (2, 3)]
        common = (t, n, h, nd, dy.data_ptr(), dy_dirs, w_hh_f.data_ptr(), _p(w_hh_r),
                  h_all.data_ptr(), gates.data_ptr(), lens.data_ptr(), dgx.data_ptr(),
                  dgh.data_ptr(), dbias[0].data_ptr(), dbias[1].data_ptr(),
                  _p(dbias[2] if nd == 2 else None), _p(dbias[3] if nd == 2 else None))
        col_amax = None
        if h3_enabled() and not bf16:
            col_amax = torch.empty(2 * nd * h3, dtype=_I32, device=dev)
            _lib.call("ds2_gru_bwd_bias_amax", *common, col_amax.data_ptr(),
                      rnn_status_word(dev).data_ptr(), ws.data_ptr(), ws.numel(), _stream())
        else:
            _lib.call("ds2_gru_bwd_bias", *common, rnn_status_word(dev).data_ptr(),
                      ws.data_ptr(), ws.numel(), _stream())
        dx, grads = _rnn_param_grads(x, h_all, dgx, dgh, weights, nd, h3,
                                     ctx.needs_input_grad[0], bf16, ctx.pre, dbias=dbias,
                                     col_amax=col_amax)
        return (dx, None, None, None, *grads)


class RNNLayerFn(torch.autograd.Function):
    """One (bi)directional vanilla tanh RNN layer (nn.RNN, rnn_type 'rnn', model.py:15) over
    padded [T, N, In] + lengths: pack -> nn.RNN -> pad of model.py:103-105; with sum_dirs the
    direction sum of model.py:107.  Input projection and every parameter gradient are the
    GRU's GEMMs with one gate; the recurrence is ds2_rnn_fwd_ws / ds2_rnn_bwd_ws (the GRU's
    persistent fp16x3 machinery with one gate; per-step kernels where it declines)."""

    @staticmethod
    def forward(ctx, x, lens, sum_dirs, hidden, *weights):
        x = x.contiguous()
        t, n, _ = x.shape
        h = hidden
        nd = len(weights) // 4
        dev = x.device
        bf16 = _RNN_GEMM_BF16[0]
        xproj, ctx.pre = _rnn_input_proj(x, weights, nd, h, bf16, ctx.needs_input_grad[0])
        h_all = torch.empty(t, n, nd, h, device=dev, dtype=_F32)
        ws = _ws(_lib.size("ds2_rnn_fwd_workspace_size", n, h, nd), dev)
        _lib.call("ds2_rnn_fwd_ws", t, n, h, nd, xproj.data_ptr(), weights[1].data_ptr(),
                  _p(weights[5] if nd == 2 else None), weights[3].data_ptr(),
                  _p(weights[7] if nd == 2 else None), lens.data_ptr(), h_all.data_ptr(),
                  rnn_status_word(dev).data_ptr(), ws.data_ptr(), ws.numel(), _stream())
        ctx.save_for_backward(x, lens, h_all, *weights)
        ctx.cfg = (sum_dirs, h, nd, bf16)
        return _rnn_output(h_all, sum_dirs, nd)

    @staticmethod
    def backward(ctx, dy):
        x, lens, h_all, *weights = ctx.saved_tensors
        sum_dirs, h, nd, bf16 = ctx.cfg
        t, n, _ = x.shape
        dy = dy.contiguous()
        dy_dirs = 1 if (sum_dirs and nd == 2) else nd
        dev = x.device
        dg = torch.empty(t, n, nd, h, device=dev, dtype=_F32)
        ws = _ws(_lib.size("ds2_rnn_bwd_workspace_size", n, h, nd), dev)
        _guard_cooperative("rnn", n, h, nd)
        col_amax = (torch.empty(nd * h, dtype=_I32, device=dev)
                    if h3_enabled() and not bf16 else None)
        _lib.call("ds2_rnn_bwd_ws", t, n, h, nd, dy.data_ptr(), dy_dirs, weights[1].data_ptr(),
                  _p(weights[5] if nd == 2 else None), h_all.data_ptr(), lens.data_ptr(),
                  dg.data_ptr(), _p(col_amax), rnn_status_word(dev).data_ptr(), ws.data_ptr(),
                  ws.numel(), _stream())
        dx, grads = _rnn_param_grads(x, h_all, dg, dg, weights, nd, h,
                                     ctx.needs_input_grad[0], bf16, ctx.pre, col_amax=col_amax)
        return (dx, None, None, None, *grads)


class LSTMLayerFn(torch.autograd.Function):
    """One (bi)directional LSTM layer (nn.LSTM semantics, gates i, f, g, o) over padded
    [T, N, In] + lengths: pack -> nn.LSTM -> pad of model.py:103-105 (rnn_type 'lstm',
    model.py:14); with sum_dirs the direction sum of model.py:107."""

    @staticmethod
    def forward(ctx, x, lens, sum_dirs, hidden, *weights):
        x = x.contiguous()
        t, n, _ = x.shape
        h = hidden
        nd = len(weights) // 4
        dev = x.device
        bf16 = _RNN_GEMM_BF16[0]
        xproj, ctx.pre = _rnn_input_proj(x, weights, nd, 4 * h, bf16, ctx.needs_input_grad[0])
        h_all = torch.empty(t, n, nd, h, device=dev, dtype=_F32)
        need_grad = any(ctx.needs_input_grad)
        c_all = torch.empty(t, n, nd, h, device=dev, dtype=_F32) if need_grad else None
        gates = torch.empty(t, n, nd, 4 * h, device=dev, dtype=_F32) if need_grad else None
        w_hh_f, b_hh_f = weights[1], weights[3]
        w_hh_r = weights[5] if nd == 2 else None
        b_hh_r = weights[7] if nd == 2 else None
        ws = _ws(_lib.size("ds2_lstm_fwd_workspace_size", n, h, nd), dev)
        _lib.call("ds2_lstm_fwd", t, n, h, nd, xproj.data_ptr(), w_hh_f.data_ptr(), _p(w_hh_r),
                  b_hh_f.data_ptr(), _p(b_hh_r), lens.data_ptr(), h_all.data_ptr(), _p(c_all),
                  _p(gates), rnn_status_word(dev).data_ptr(), ws.data_ptr(), ws.numel(), _stream())
        ctx.save_for_backward(x, lens, h_all, c_all, gates, *weights)
        ctx.cfg = (sum_dirs, h, nd, bf16)
        return _rnn_output(h_all, sum_dirs, nd)

    @staticmethod
    def backward(ctx, dy):
        x, lens, h_all, c_all, gates, *weights = ctx.saved_tensors
        sum_dirs, h, nd, bf16 = ctx.cfg
        t, n, _ = x.shape
        dev = x.device
        dy = dy.contiguous()
        dy_dirs = 1 if (sum_dirs and nd == 2) else nd
        dg = torch.empty(t, n, nd, 4 * h, device=dev, dtype=_F32)
        w_hh_f = weights[1]
        w_hh_r = weights[5] if nd == 2 else None
        ws = _ws(_lib.size("ds2_lstm_bwd_workspace_size", n, h, nd), dev)
        # bf16 mode (BASELINE cfg4): the recurrence's W_hh^T product on one fp16 term too
        half = bf16 and os.environ.get("DS2_LSTM_HALF", "1")[:1] != "0"
        _guard_cooperative("lstm_half" if half else "lstm", n, h, nd)
        _lib.call("ds2_lstm_bwd_half" if half else "ds2_lstm_bwd", t, n, h, nd, dy.data_ptr(),
                  dy_dirs, w_hh_f.data_ptr(),
                  _p(w_hh_r), c_all.data_ptr(), gates.data_ptr(), lens.data_ptr(), dg.data_ptr(),
                  rnn_status_word(dev).data_ptr(), ws.data_ptr(), ws.numel(), _stream())
        dx, grads = _rnn_param_grads(x, h_all, dg, dg, weights, nd, 4 * h,
                                     ctx.needs_input_grad[0], bf16, ctx.pre)
        return (dx, None, None, None, *grads)


class LookaheadFn(torch.autograd.Function):
    """Lookahead conv (model.py:140-177) on [T, N, H], optionally fused with the
    Hardtanh(lo, hi) that follows it in DeepSpeech (model.py:329-333)."""

    @staticmethod
    def forward(ctx, x, weight, clamp):
        x = _need(x, "lookahead x").contiguous()
        w = _need(weight, "lookahead weight").contiguous()
        t, n, h = x.shape
        context = w.shape[1] - 1
        y = torch.empty_like(x)
        lo, hi = clamp if clamp is not None else (0.0, 0.0)
        _lib.call("ds2_lookahead_fwd", x.data_ptr(), t, n, h, w.data_ptr(), context,
                  int(clamp is not None), lo, hi, y.data_ptr(), _stream())
        ctx.save_for_backward(x, w, y if clamp is not None else None)
        ctx.clamp = clamp
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        t, n, h = x.shape
        context = w.shape[1] - 1
        lo, hi = ctx.clamp if ctx.clamp is not None else (0.0, 0.0)
        dy = dy.contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw = grad_like(w) if ctx.needs_input_grad[1] else None
        ws = _ws(_lib.size("ds2_lookahead_bwd_workspace_size", t, n, h, context), x.device)
        _lib.call("ds2_lookahead_bwd", dy.data_ptr(), _p(y), lo, hi, x.data_ptr(), t, n, h,
                  w.data_ptr(), context, _p(dx), _p(dw), ws.data_ptr(), ws.numel(), _stream())
        return dx, dw, None


class CTCLossFn(torch.autograd.Function):
    """warp-ctc semantics: summed cost, gradient wrt pre-softmax activations."""

    @staticmethod
    def forward(ctx, acts, labels, act_lens, label_lens, max_label_len, blank, zero_infinity,
                size_average):
        costs, grads = ctc_loss_raw(acts, labels, act_lens, label_lens, max_label_len, blank,
                                    zero_infinity, want_grad=True)
        loss = costs.sum()
        if size_average:
            n = acts.shape[1]
            loss = loss / n
            grads.mul_(1.0 / n)
        ctx.save_for_backward(grads)
        return loss

    @staticmethod
    def backward(ctx, grad_out):
        (grads,) = ctx.saved_tensors
        g = grads.clone()
        go = grad_out.reshape(1).to(dtype=_F32).contiguous()
        _lib.call("ds2_scale_by_device_scalar", g.data_ptr(), g.numel(), go.data_ptr(), _stream())
        return g, None, None, None, None, None, None, None


class SoftmaxTNCFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits_tnc):
        probs = softmax_tnc(logits_tnc)
        ctx.save_for_backward(probs)
        return probs

    @staticmethod
    def backward(ctx, dprobs):
        (probs,) = ctx.saved_tensors
        n, t, c = probs.shape
        d = torch.empty(t, n, c, device=probs.device, dtype=_F32)
        _lib.call("ds2_softmax_tnc_bwd", probs.data_ptr(), dprobs.contiguous().data_ptr(), t, n, c,
                  d.data_ptr(), 0, _stream())
        return d
