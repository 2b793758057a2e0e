"""CPU restatement of the librosa / resampy pieces the reference's waveform augmentations
call — TEST INFRASTRUCTURE (the checker for ds2_time_stretch / ds2_resample).

The reference calls them positionally (librosa < 0.10):
  * ChangeAudioSpeed: ``librosa.effects.time_stretch(wav, alpha)``  (data/audio_aug.py:7-23)
  * PitchShift: ``librosa.effects.pitch_shift(wav, sr, n_steps=alpha)``  (:63-75)
  * a file at another sample rate: ``librosa.resample(y, sr_file, sr)``
    (data/data_loader_aug.py:668; res_type 'kaiser_best' = resampy)

librosa and resampy are NOT installed here, so these are restatements of their published
algorithms, pinned in tests/test_librosa_effects.py by analytic known answers (a tone keeps
its frequency through time_stretch, pitch_shift moves it by 2**(n/12), resampling preserves a
band-limited tone, lengths follow the formulas below) — parity with librosa / resampy
themselves is UNPINNED.  Versions restated: librosa 0.8.x (stft center=True, pad_mode
'reflect', n_fft 2048, hop n_fft // 4, periodic Hann window; phase_vocoder; istft with
``length``; window_sumsquare normalisation) and resampy 0.2.x (``resample_f``; 'kaiser_best'
= ``sinc_window(num_zeros=64, precision=9, window=kaiser(beta=14.769656459379492),
rolloff=0.9475937167399596)``).  dtypes follow numpy 1.x's rules for a float32 input: the stft
matrix is complex64, the vocoder's magnitude interpolation float32, the vocoder's phase accumulator float32, the overlap-add buffer and the
window sum float32 (every add rounded), resampy accumulates every tap into its float32 output.
"""
from __future__ import annotations

import numpy as np

N_FFT = 2048
HOP = N_FFT // 4


def hann_periodic(n: int) -> np.ndarray:
    """scipy.signal.get_window('hann', n, fftbins=True): scipy's general_cosine over n + 1
    points, last one dropped -- the same float64 operations, since the vocoder's float32 phase
    accumulator turns even a one-ulp (2e-16) change of the window into a ~7e-5 (of peak)
    change of the stretched signal."""
    fac = np.linspace(-np.pi, np.pi, n + 1)
    w = np.zeros(n + 1)
    w += 0.5 * np.cos(0 * fac)
    w += 0.5 * np.cos(fac)
    return w[:-1]


def stft(y: np.ndarray, n_fft: int = N_FFT, hop: int = HOP) -> np.ndarray:
    """librosa.stft(y) (0.8): reflect-pad n_fft // 2, frames of n_fft every hop, periodic
    Hann, fft in float64 stored complex64 -> [1 + n_fft // 2, frames]."""
    y = np.asarray(y)
    yp = np.pad(y, n_fft // 2, mode='reflect')
    n_frames = 1 + (len(yp) - n_fft) // hop
    idx = np.arange(n_fft)[:, None] + hop * np.arange(n_frames)[None, :]
    frames = hann_periodic(n_fft)[:, None] * yp[idx]
    return np.fft.fft(frames, axis=0)[:1 + n_fft // 2].astype(np.complex64)


# numpy's float32 np.abs / np.angle / np.exp(1j * x) of a complex64 are platform-dependent in
# their last bits (libm hypotf / atan2f / sincosf, or SVML-based SIMD loops on AVX-512 hosts),
# and the vocoder's float32 phase accumulator (which grows to ~1e4 rad in the high bins) turns a
# one-ulp difference of an angle into a visibly different rounding.  The restatement fixes them
# to their correctly rounded values (evaluated in float64, rounded once to float32).
def _absf(c: np.ndarray) -> np.ndarray:
    re, im = c.real.astype(np.float64), c.imag.astype(np.float64)
    return np.sqrt(re * re + im * im).astype(np.float32)


def _anglef(c: np.ndarray) -> np.ndarray:
    return np.arctan2(c.imag.astype(np.float64), c.real.astype(np.float64)).astype(np.float32)


def _expjf(x: np.ndarray) -> np.ndarray:
    xd = x.astype(np.float64)
    return (np.cos(xd).astype(np.float32) + 1j * np.sin(xd).astype(np.float32)).astype(np.complex64)


def phase_vocoder(D: np.ndarray, rate: float, hop: int = HOP) -> np.ndarray:
    """librosa.phase_vocoder(D, rate) (0.8)."""
    time_steps = np.arange(0, D.shape[1], rate, dtype=np.float64)
    out = np.zeros((D.shape[0], len(time_steps)), D.dtype, order='F')
    phi_advance = np.linspace(0, np.pi * hop, D.shape[0])
    phase_acc = _anglef(D[:, 0])                       # float32 for complex64 D
    D = np.pad(D, [(0, 0), (0, 2)], mode='constant')
    for t, step in enumerate(time_steps):
        cols = D[:, int(step):int(step + 2)]
        alpha = np.mod(step, 1.0)
        # numpy 1.x (the reference's era) value-based casting: the float64 scalars (1 - alpha),
        # alpha meet the float32 magnitudes in float32; stated explicitly so numpy 2 agrees
        mag = np.float32(1.0 - alpha) * _absf(cols[:, 0]) + np.float32(alpha) * _absf(cols[:, 1])
        e = _expjf(phase_acc)                          # complex64 (cos, sin) of the float32 phase
        out[:, t] = (mag * e.real).astype(np.float32) + 1j * (mag * e.imag).astype(np.float32)
        dphase = (_anglef(cols[:, 1]) - _anglef(cols[:, 0])) - phi_advance
        dphase = dphase - 2.0 * np.pi * np.round(dphase / (2.0 * np.pi))
        phase_acc += phi_advance + dphase
    return out


def istft(D: np.ndarray, length: int, dtype=np.float32, hop: int = HOP) -> np.ndarray:
    """librosa.istft(D, dtype=dtype, length=length) (0.8, center=True, periodic Hann)."""
    n_fft = 2 * (D.shape[0] - 1)
    win = hann_periodic(n_fft)
    n_frames = min(D.shape[1], int(np.ceil((length + n_fft) / hop)))
    total = n_fft + hop * (n_frames - 1)
    y = np.zeros(total, dtype=dtype)
    for i in range(n_frames):
        ytmp = win * np.fft.irfft(D[:, i], n=n_fft)
        y[i * hop:i * hop + n_fft] += ytmp              # rounded to dtype per frame
    wss = np.zeros(total, dtype=dtype)
    win_sq = win ** 2
    for i in range(n_frames):
        wss[i * hop:i * hop + n_fft] += win_sq          # window_sumsquare, dtype adds
    nz = wss > np.finfo(wss.dtype).tiny
    y[nz] /= wss[nz]
    y = y[n_fft // 2:]
    out = np.zeros(length, dtype=dtype)
    k = min(length, len(y))
    out[:k] = y[:k]
    return out


def stretch_length(n: int, rate: float) -> int:
    """len(time_stretch(y, rate)) = int(round(len(y) / rate))."""
    return int(round(n / rate))


def time_stretch(y: np.ndarray, rate: float) -> np.ndarray:
    """librosa.effects.time_stretch(y, rate) (0.8)."""
    if rate <= 0:
        raise ValueError("rate must be a positive number")
    D = phase_vocoder(stft(y), rate)
    return istft(D, stretch_length(len(y), rate), dtype=y.dtype)


def time_stretch_f64(y: np.ndarray, rate: float) -> np.ndarray:
    """The same STFT -> phase vocoder -> ISTFT chain with every intermediate in float64 (no
    float32 rounding of the stft matrix, magnitudes, phase accumulator or overlap-add): the
    yardstick for the float32 phase noise librosa's own chain carries (tests compare the
    device's distance from the restatement against the restatement's distance from this)."""
    y = np.asarray(y, dtype=np.float64)
    yp = np.pad(y, N_FFT // 2, mode='reflect')
    n_frames = 1 + (len(yp) - N_FFT) // HOP
    idx = np.arange(N_FFT)[:, None] + HOP * np.arange(n_frames)[None, :]
    D = np.fft.rfft(hann_periodic(N_FFT)[:, None] * yp[idx], axis=0)
    steps = np.arange(0, D.shape[1], rate, dtype=np.float64)
    phi = np.linspace(0, np.pi * HOP, D.shape[0])
    acc = np.angle(D[:, 0])
    Dp = np.pad(D, [(0, 0), (0, 2)])
    V = np.zeros((D.shape[0], len(steps)), complex)
    for t, st in enumerate(steps):
        c = Dp[:, int(st):int(st) + 2]
        a = np.mod(st, 1.0)
        V[:, t] = ((1 - a) * np.abs(c[:, 0]) + a * np.abs(c[:, 1])) * np.exp(1j * acc)
        dp = np.angle(c[:, 1]) - np.angle(c[:, 0]) - phi
        dp = dp - 2.0 * np.pi * np.round(dp / (2.0 * np.pi))
        acc = acc + phi + dp
    return istft(V, stretch_length(len(y), rate), dtype=np.float64)


# ------------------------------------------------------------------------------ resampy
KAISER_BEST = dict(num_zeros=64, precision=9, beta=14.769656459379492,
                   rolloff=0.9475937167399596)


def kaiser_best_filter():
    """resampy.filters.sinc_window(64, 9, kaiser(beta=14.7697), 0.9476): the right wing of
    a Kaiser-windowed sinc sampled 2**9 times per zero crossing -> (interp_win, 512)."""
    from scipy.signal.windows import kaiser
    p = KAISER_BEST
    num_bits = 2 ** p['precision']
    n = num_bits * p['num_zeros']
    sinc_win = p['rolloff'] * np.sinc(p['rolloff'] * np.linspace(0, p['num_zeros'], num=n + 1,
                                                                  endpoint=True))
    taper = kaiser(2 * n + 1, p['beta'])[n:]
    return taper * sinc_win, num_bits


def resample_length(n: int, sr_orig, sr_new) -> int:
    """resampy's output length int(n * sr_new / sr_orig)."""
    return int(n * (float(sr_new) / sr_orig))


def resampy_resample(x: np.ndarray, sr_orig, sr_new) -> np.ndarray:
    """resampy.resample(x, sr_orig, sr_new, filter='kaiser_best') (0.2, resample_f) for a
    1-D float32 signal: windowed-sinc interpolation, every tap accumulated into the float32
    output element in the loop order below."""
    ratio = float(sr_new) / sr_orig
    n_out = int(x.shape[0] * ratio)
    y = np.zeros(n_out, dtype=x.dtype)
    win, num_table = kaiser_best_filter()
    if ratio < 1:
        win = win * ratio
    delta = np.zeros_like(win)
    delta[:-1] = np.diff(win)
    scale = min(1.0, ratio)
    time_increment = 1.0 / ratio
    index_step = int(scale * num_table)
    nwin = win.shape[0]
    n_orig = x.shape[0]
    xd = x.astype(np.float64)
    # time_register += time_increment once per output sample (sequential, as np.add.accumulate)
    treg = np.zeros(n_out, dtype=np.float64)
    if n_out > 1:
        treg[1:] = np.add.accumulate(np.full(n_out - 1, time_increment))
    n = treg.astype(np.int64)
    acc = np.zeros(n_out, dtype=np.float32)
    for wing in (0, 1):
        frac = scale * (treg - n)
        if wing:
            frac = scale - frac
        index_frac = frac * num_table
        offset = index_frac.astype(np.int64)
        eta = index_frac - offset
        if wing == 0:
            cnt = np.minimum(n + 1, (nwin - offset) // index_step)
        else:
            cnt = np.minimum(n_orig - n - 1, (nwin - offset) // index_step)
        for i in range(int(cnt.max()) if n_out else 0):
            m = cnt > i
            j = offset[m] + i * index_step
            w = win[j] + eta[m] * delta[j]
            src = n[m] - i if wing == 0 else n[m] + i + 1
            acc[m] = (acc[m].astype(np.float64) + w * xd[src]).astype(np.float32)
    y[:] = acc
    return y


def resample(y: np.ndarray, orig_sr, target_sr) -> np.ndarray:
    """librosa.resample(y, orig_sr, target_sr) (0.8; res_type 'kaiser_best', fix=True):
    resampy, then fix_length to ceil(len * ratio)."""
    if orig_sr == target_sr:
        return y
    ratio = float(target_sr) / orig_sr
    n_samples = int(np.ceil(y.shape[-1] * ratio))
    y_hat = resampy_resample(y, orig_sr, target_sr)
    out = np.zeros(n_samples, dtype=y_hat.dtype)
    k = min(n_samples, len(y_hat))
    out[:k] = y_hat[:k]
    return out


def pitch_rate(n_steps: float, bins_per_octave: int = 12) -> float:
    return 2.0 ** (-float(n_steps) / bins_per_octave)


def pitch_shift(y: np.ndarray, sr, n_steps: float) -> np.ndarray:
    """librosa.effects.pitch_shift(y, sr, n_steps) (0.8): time_stretch by
    rate = 2 ** (-n_steps / 12), resample sr / rate -> sr, fix_length to len(y)."""
    rate = pitch_rate(n_steps)
    y_shift = resample(time_stretch(y, rate), float(sr) / rate, sr)
    out = np.zeros(len(y), dtype=y_shift.dtype)
    k = min(len(y), len(y_shift))
    out[:k] = y_shift[:k]
    return out


def dominant_frequency(y: np.ndarray, sr: float) -> float:
    """Peak of |rfft| of a Hann-windowed signal with parabolic interpolation (test helper)."""
    w = np.hanning(len(y))
    s = np.abs(np.fft.rfft(y * w))
    k = int(np.argmax(s[1:-1])) + 1
    a, b, c = np.log(s[k - 1] + 1e-30), np.log(s[k] + 1e-30), np.log(s[k + 1] + 1e-30)
    p = 0.5 * (a - c) / (a - 2 * b + c)
    return (k + p) * sr / len(y)

