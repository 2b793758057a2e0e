"""ctypes binding of libds2hip.so (the C ABI declared in include/ds2hip.h).

The shared library is built in-tree (``deepspeech.pytorch_amd/csrc/Makefile``)
and loaded from this directory.  There is no fallback: if the library is
missing every GPU op raises, so a silently slower path can never stand in for
the HIP kernels.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DS2_LIB_PATH") or os.path.join(_HERE, "libds2hip.so")

_c_int = ctypes.c_int
_c_i64 = ctypes.c_int64
_c_f = ctypes.c_float
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t

# name -> (restype, argtypes)
_PROTOS = {
    "ds2_status_string": (ctypes.c_char_p, [_c_int]),
    "ds2_last_error": (ctypes.c_char_p, []),
    "ds2_version": (ctypes.c_char_p, []),
    "ds2_stft_workspace_size": (_sz, [_c_int, _c_int, _c_int]),
    "ds2_stft_logmag": (_c_int, [_vp, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _vp,
                                 _c_int, _vp, _c_int, _vp, _sz, _vp]),
    "ds2_stft_logmag_masked": (_c_int, [_vp, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _c_int,
                                        _vp, _c_int, _vp, _vp, _c_int, _vp, _sz, _vp]),
    "ds2_wave_aug_workspace_size": (_sz, [_c_int, _c_i64]),
    "ds2_wave_aug": (_c_int, [_vp, _c_i64, _vp, _c_int, _vp, _vp, _c_int, _vp, _c_i64, _vp,
                              _c_i64, _vp, _c_i64, _vp, _vp, _sz, _vp]),
    "ds2_time_stretch_workspace_size": (_sz, [_c_int, _c_int, _c_int]),
    "ds2_time_stretch": (_c_int, [_vp, _c_i64, _vp, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _c_i64,
                                  _c_int, _c_int, _vp, _sz, _vp]),
    "ds2_resample_workspace_size": (_sz, [_c_int, _c_i64]),
    "ds2_resample": (_c_int, [_vp, _c_i64, _vp, _c_int, _vp, _vp, _vp, _c_int, _c_int, _vp,
                              _c_i64, _vp, _sz, _vp]),
    "ds2_sgemm": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_f, _vp, _c_i64, _c_i64,
                           _vp, _c_i64, _c_i64, _c_f, _vp, _c_i64, _c_i64, _c_int, _vp, _vp]),
    "ds2_sgemm_workspace_size": (_sz, [_c_int, _c_int, _c_int, _c_int]),
    "ds2_sgemm_ws": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_f, _vp, _c_i64, _c_i64,
                              _vp, _c_i64, _c_i64, _c_f, _vp, _c_i64, _c_i64, _c_int, _vp, _vp,
                              _sz, _vp]),
    "ds2_sgemm_bf16_workspace_size": (_sz, [_c_int, _c_int, _c_int, _c_int]),
    "ds2_sgemm_bf16_ws": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_f, _vp, _c_i64,
                                   _c_i64, _vp, _c_i64, _c_i64, _c_f, _vp, _c_i64, _c_i64, _c_int,
                                   _vp, _vp, _sz, _vp]),
    "ds2_conv2d_workspace_size": (_sz, [_c_int] * 11),
    "ds2_conv2d_fwd": (_c_int, [_vp, _vp, _vp, _vp] + [_c_int] * 11 + [_vp, _vp, _sz, _vp]),
    "ds2_conv2d_dgrad": (_c_int, [_vp, _vp, _vp] + [_c_int] * 11 + [_vp, _sz, _vp]),
    "ds2_conv2d_wgrad_workspace_size": (_sz, [_c_int] * 11),
    "ds2_conv2d_wgrad": (_c_int, [_vp, _vp, _vp, _vp] + [_c_int] * 11 + [_vp, _sz, _vp]),
    "ds2_bn_workspace_size": (_sz, [_c_int, _c_int, _c_int]),
    "ds2_bn_train_stats": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_f, _c_f, _vp, _vp, _vp, _vp,
                                    _vp, _sz, _vp]),
    "ds2_bn_eval_stats": (_c_int, [_vp, _vp, _c_int, _c_f, _vp, _vp, _vp]),
    "ds2_bn_apply": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _vp]),
    "ds2_bn_apply_amax": (_c_int, [_vp, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "ds2_bn_apply_mask_htanh": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp,
                                         _vp, _c_f, _c_f, _vp, _c_int, _vp]),
    "ds2_bn_backward": (_c_int, [_vp, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp,
                                 _vp, _c_int, _vp, _c_f, _c_f, _vp, _vp, _vp, _vp, _vp, _sz,
                                 _vp]),
    "ds2_gru_fwd_workspace_size": (_sz, [_c_int, _c_int, _c_int]),
    "ds2_gru_cache_floats": (_sz, [_c_int, _c_int, _c_int, _c_int]),
    "ds2_gru_fwd": (_c_int, [_c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                             _vp, _vp, _vp, _sz, _vp]),
    "ds2_gru_bwd_workspace_size": (_sz, [_c_int, _c_int, _c_int]),
    "ds2_gru_bwd_grid": (_c_int, [_c_int, _c_int, _c_int]),
    "ds2_lstm_bwd_grid": (_c_int, [_c_int, _c_int, _c_int]),
    "ds2_bgemm_workspace_size": (_sz, [_c_int, _c_int, _c_int]),
    "ds2_bgemm_nt": (_c_int, [_c_int, _c_int, _c_int, _c_f, _vp, _c_i64, _vp, _c_i64, _c_f, _vp,
                              _c_i64, _vp, _vp, _sz, _vp]),
    "ds2_cvt_bf16": (_c_int, [_vp, _c_int, _c_int, _c_i64, _vp, _c_i64, _c_int, _vp]),
    "ds2_rnn_fwd": (_c_int, [_c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                             _vp]),
    "ds2_rnn_bwd": (_c_int, [_c_int, _c_int, _c_int, _c_int, _vp, _c_int, _vp, _vp, _vp, _vp,
                             _vp, _vp]),
    "ds2_rnn_fwd_workspace_size": (_sz, [_c_int, _c_int, _c_int]),
    "ds2_rnn_fwd_ws": (_c_int, [_c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                _vp, _vp, _sz, _vp]),
    "ds2_rnn_bwd_workspace_size": (_sz, [_c_int, _c_int, _c_int]),
    "ds2_rnn_bwd_grid": (_c_int, [_c_int, _c_int, _c_int]),
    "ds2_rnn_bwd_ws": (_c_int, [_c_int, _c_int, _c_int, _c_int, _vp, _c_int, _vp, _vp, _vp, _vp,
                                _vp, _vp, _vp, _vp, _sz, _vp]),
    "ds2_test_occupy": (_c_int, [_c_int, _c_int, _c_int, _vp, _vp]),
    "ds2_test_rnn_launch_lds": (_c_int, [_c_int, _c_int, _vp, _vp]),
    "ds2_test_timestamp": (_c_int, [_vp, _vp]),
    "ds2_amax": (_c_int, [_vp, _c_int, _c_int, _c_i64, _vp, _vp, _vp]),
    "ds2_sgemm_amax_ws": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_f, _vp, _c_i64, _vp,
                                   _c_i64, _c_f, _vp, _c_i64, _vp, _vp, _vp, _vp, _sz, _vp]),
    "ds2_test_ring_traffic": (_c_int, [_vp, _c_i64, _c_int, _vp, _c_int, ctypes.c_double, _vp]),
    "ds2_test_beam_stamps": (_c_int, [_vp]),
    "ds2_gru_bwd": (_c_int, [_c_int, _c_int, _c_int, _c_int, _vp, _c_int, _vp, _vp, _vp, _vp,
                             _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "ds2_gru_bwd_bias": (_c_int, [_c_int, _c_int, _c_int, _c_int, _vp, _c_int, _vp, _vp, _vp,
                                  _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "ds2_gru_bwd_bias_amax": (_c_int, [_c_int, _c_int, _c_int, _c_int, _vp, _c_int, _vp, _vp,
                                       _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                       _sz, _vp]),
    "ds2_lstm_fwd_workspace_size": (_sz, [_c_int, _c_int, _c_int]),
    "ds2_lstm_fwd": (_c_int, [_c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                              _vp, _vp, _vp, _vp, _sz, _vp]),
    "ds2_lstm_bwd_workspace_size": (_sz, [_c_int, _c_int, _c_int]),
    "ds2_lstm_bwd": (_c_int, [_c_int, _c_int, _c_int, _c_int, _vp, _c_int, _vp, _vp, _vp, _vp,
                              _vp, _vp, _vp, _vp, _sz, _vp]),
    "ds2_lstm_bwd_half_grid": (_c_int, [_c_int, _c_int, _c_int]),
    "ds2_lstm_bwd_half": (_c_int, [_c_int, _c_int, _c_int, _c_int, _vp, _c_int, _vp, _vp, _vp,
                                   _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "ds2_lookahead_fwd": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _c_int, _c_int, _c_f,
                                   _c_f, _vp, _vp]),
    "ds2_lookahead_bwd_workspace_size": (_sz, [_c_int, _c_int, _c_int, _c_int]),
    "ds2_lookahead_bwd": (_c_int, [_vp, _vp, _c_f, _c_f, _vp, _c_int, _c_int, _c_int, _vp,
                                   _c_int, _vp, _vp, _vp, _sz, _vp]),
    "ds2_dirsum": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp]),
    "ds2_colsum_workspace_size": (_sz, [_c_int, _c_int]),
    "ds2_colsum": (_c_int, [_vp, _c_int, _c_int, _c_i64, _vp, _c_int, _vp, _sz, _vp]),
    "ds2_softmax_tnc": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp]),
    "ds2_softmax_tnc_bwd": (_c_int, [_vp, _vp, _c_int, _c_int, _c_int, _vp, _c_int, _vp]),
    "ds2_ctc_workspace_size": (_sz, [_c_int, _c_int, _c_int]),
    "ds2_ctc_loss": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp, _vp, _c_int, _c_int, _c_int,
                              _vp, _vp, _vp, _sz, _vp]),
    "ds2_greedy_decode": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_i64, _c_i64, _vp, _c_int, _vp,
                                   _vp, _vp, _vp, _vp]),
    "ds2_edit_distance": (_c_int, [_vp, _c_i64, _vp, _vp, _vp, _vp, _c_int, _c_int, _vp, _vp,
                                   _vp]),
    "ds2_ctc_beam_workspace_size": (_sz, [_c_int, _c_int, _c_int]),
    "ds2_ctc_beam_decode": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_i64, _c_i64, _vp, _c_int,
                                     _c_int, _c_int, ctypes.c_double, _c_int, _vp, _vp, _vp, _vp,
                                     _vp, _sz, _vp]),
    "ds2_ctc_beam_decode_lm": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_i64, _c_i64, _vp, _c_int,
                                        _c_int, _c_int, ctypes.c_double, _c_int, _c_int, _c_int,
                                        _c_int, _c_int, ctypes.c_double, ctypes.c_double, _vp, _vp,
                                        _vp, _c_int, _c_int, _vp, _c_i64, _vp, _vp, _vp, _vp, _vp,
                                        _sz, _vp]),
    "ds2_comm_id_bytes": (_sz, []),
    "ds2_comm_get_unique_id": (_c_int, [_vp]),
    "ds2_comm_init": (_c_int, [_vp, _vp, _c_int, _c_int, _c_int]),
    "ds2_allreduce_bucket": (_c_int, [_vp, _vp, _c_i64, _vp]),
    "ds2_comm_destroy": (_c_int, [_vp]),
    "ds2_optim_workspace_size": (_sz, [_c_i64]),
    "ds2_grad_norm": (_c_int, [_vp, _c_i64, _vp, _vp, _sz, _vp]),
    "ds2_clip_sgd_nesterov": (_c_int, [_vp, _vp, _vp, _c_i64, _c_f, _c_f, _c_f, _vp, _vp, _vp]),
    "ds2_nan_guard": (_c_int, [_vp, _c_i64, _c_int, _vp, _vp, _vp]),
    "ds2_zero_masked": (_c_int, [_vp, _vp, _c_i64, _vp, _vp]),
    "ds2_scale_by_device_scalar": (_c_int, [_vp, _c_i64, _vp, _vp]),
}

EXPORTED_SYMBOLS = tuple(_PROTOS)

_lock = threading.Lock()
_lib = None


class Ds2Error(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load libds2hip.so once; raises Ds2Error when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise Ds2Error(
                f"libds2hip.so not found at {LIB_PATH}; build it with "
                "`make -C deepspeech.pytorch_amd/csrc` (or __graft_entry__.build()). "
                "There is no CPU fallback for the product path.")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _PROTOS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(status: int, what: str) -> None:
    if status != 0:
        lib = load()
        msg = lib.ds2_status_string(status).decode()
        last = lib.ds2_last_error().decode()
        raise Ds2Error(f"{what} failed: {msg}" + (f" ({last})" if last else ""))


def call(name: str, *args) -> None:
    lib = load()
    check(getattr(lib, name)(*args), name)


def size(name: str, *args) -> int:
    return int(getattr(load(), name)(*args))
