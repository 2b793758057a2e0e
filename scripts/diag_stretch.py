"""Diagnostic: where does the device time_stretch differ from the oracle restatement?
usage: python scripts/diag_stretch.py  (GPU)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ds2amd import ops  # noqa: E402
from oracle import librosa_effects as le  # noqa: E402
from tests.test_librosa_effects import _speech_like  # noqa: E402

dev = torch.device("cuda")
for n, r, seed in ((16000, 0.85, 0), (16000, 1.0, 0), (9001, 1.15, 1), (4096, 1.0, 3)):
    y = _speech_like(n, seed)
    out, ol = ops.time_stretch(torch.from_numpy(y)[None].to(dev), [n], [r])
    d = out[0, :ol[0]].cpu().numpy()
    e = le.time_stretch(y, r)
    err = np.abs(d - e)
    peak = np.abs(e).max()
    i = int(err.argmax())
    blk = [float(err[k:k + 512].max() / peak) for k in range(0, len(e), 512)]
    print(f"n {n} rate {r}: len {len(e)} max rel {err.max() / peak:.3e} at {i}; per-512 block:",
          " ".join(f"{b:.1e}" for b in blk[:12]), "...", " ".join(f"{b:.1e}" for b in blk[-4:]))
    # oracle stages with the device's (scipy-form) window
    D = le.stft(y)
    Dv = le.phase_vocoder(D, r)
    print("   stft |D| max", float(np.abs(D).max()), "vocoder frames", Dv.shape)
    # fp64 reference of the same algorithm (no float32 rounding anywhere)
    yp = np.pad(y.astype(np.float64), 1024, mode='reflect')
    nf = 1 + (len(yp) - 2048) // 512
    idx = np.arange(2048)[:, None] + 512 * np.arange(nf)[None, :]
    D64 = np.fft.fft(le.hann_periodic(2048)[:, None] * yp[idx], axis=0)[:1025]
    ts = np.arange(0, D64.shape[1], r, dtype=np.float64)
    phi = np.linspace(0, np.pi * 512, 1025)
    acc = np.angle(D64[:, 0])
    D64p = np.pad(D64, [(0, 0), (0, 2)])
    V = np.zeros((1025, len(ts)), complex)
    for t, st in enumerate(ts):
        c = D64p[:, int(st):int(st) + 2]
        a = np.mod(st, 1.0)
        V[:, t] = ((1 - a) * np.abs(c[:, 0]) + a * np.abs(c[:, 1])) * np.exp(1j * acc)
        dp = np.angle(c[:, 1]) - np.angle(c[:, 0]) - phi
        dp = dp - 2 * np.pi * np.round(dp / (2 * np.pi))
        acc = acc + phi + dp
    y64 = le.istft(V, len(e), dtype=np.float64)
    print(f"   vs fp64 algorithm: device {np.abs(d - y64).max() / peak:.3e}, oracle {np.abs(e - y64).max() / peak:.3e}")
