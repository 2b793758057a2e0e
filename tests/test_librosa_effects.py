"""librosa effects of the reference's augmentations (ChangeAudioSpeed, PitchShift, file
resampling): the oracle restatement (oracle/librosa_effects.py) pinned by analytic known
answers on CPU — librosa / resampy are absent, so parity with them is unpinned — and the
device kernels (ds2_time_stretch / ds2_resample, csrc/effects.hip) against the oracle on
the GPU, alone and inside the augmented front-end."""
import random

import numpy as np
import pytest
import torch

from ds2amd import audio_aug as aa
from ds2amd import ops
from oracle import audio_aug as oaa
from oracle import ds2_oracle as orc
from oracle import librosa_effects as le

SR = 16000


def _tone(n, f=440.0, amp=0.5, sr=SR):
    # a cosine: its reflect padding continues it smoothly (a sine's would not)
    return (amp * np.cos(2 * np.pi * f * np.arange(n) / sr)).astype(np.float32)


def _speech_like(n, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / SR
    y = sum(a * np.cos(2 * np.pi * f * t + p) for a, f, p in
            zip(rng.uniform(0.05, 0.3, 6), rng.uniform(80, 3500, 6), rng.uniform(0, 6, 6)))
    y = y * (0.6 + 0.4 * np.sin(2 * np.pi * 3 * t)) + 0.02 * rng.standard_normal(n)
    return (y / np.abs(y).max()).astype(np.float32)


# ------------------------------------------------------------------------- oracle pins (CPU)
@pytest.mark.parametrize("rate", [0.85, 0.891, 1.0, 1.07, 1.15])
def test_oracle_time_stretch_known_answers(rate):
    """A steady tone keeps its frequency and amplitude; the length is round(len / rate)."""
    y = _tone(2 * SR + 123)
    z = le.time_stretch(y, rate)
    assert z.dtype == np.float32 and len(z) == int(round(len(y) / rate))
    mid = z[4096:-4096]
    assert abs(le.dominant_frequency(mid, SR) - 440.0) < 0.05
    assert abs(np.abs(mid).max() - 0.5) < 2e-3
    if rate == 1.0:     # identity up to the float32 phase accumulator's rounding (librosa's)
        assert np.abs(z[1024:-1024] - y[1024:-1024]).max() < 2e-3


@pytest.mark.parametrize("n_steps", [-2.0, -0.7, 1.3, 2.0])
def test_oracle_pitch_shift_known_answers(n_steps):
    """The tone moves to 440 * 2^(n/12) at unchanged length and amplitude."""
    y = _tone(2 * SR)
    z = le.pitch_shift(y, SR, n_steps)
    assert len(z) == len(y)
    mid = z[4096:-4096]
    assert abs(le.dominant_frequency(mid, SR) - 440.0 * 2 ** (n_steps / 12)) < 0.05
    assert abs(np.abs(mid).max() - 0.5) < 3e-3


@pytest.mark.parametrize("sr_in,sr_out", [(8000, 16000), (22050, 16000), (16000, 8000),
                                          (44100, 16000)])
def test_oracle_resample_known_answers(sr_in, sr_out):
    """librosa.resample keeps an in-band tone (frequency; amplitude within resampy's own
    gain error: when downsampling it steps the filter table by int(ratio * 512), truncated,
    so the taps sum to ~(ratio * 512) / int(ratio * 512), +0.4 % at 44.1 -> 16 kHz); the
    length is ceil(len * sr_out / sr_in)."""
    y = _tone(sr_in, 440.0, 0.5, sr_in)
    z = le.resample(y, sr_in, sr_out)
    assert len(z) == int(np.ceil(len(y) * sr_out / sr_in))
    mid = z[1000:-1000]
    assert abs(le.dominant_frequency(mid, sr_out) - 440.0) < 0.02
    r = sr_out / sr_in
    gain = (r * 512) / int(r * 512) if r < 1 else 1.0
    assert abs(np.abs(mid).max() - 0.5 * gain) < 1e-3


def test_host_tables_match_scipy():
    """The device's window and filter tables are the ones scipy / the restatement build."""
    from scipy.signal import get_window
    assert np.array_equal(ops.hann_periodic(2048), get_window('hann', 2048, fftbins=True))
    w1, n1 = le.kaiser_best_filter()
    w2, n2 = ops.kaiser_best_filter()
    assert n1 == n2 == 512 and np.array_equal(w1, w2)
    assert w2.shape == (64 * 512 + 1,)


def test_stretch_and_pitch_records_follow_reference_draws():
    """ChangeAudioSpeed / PitchShift in the aug_type-0 OneOf: the same random / np.random
    sequence as the oracle (final states equal), the same output lengths, the records."""
    wavs = [_speech_like(int(n), i) for i, n in enumerate(np.linspace(3000, 9000, 30))]
    ours = aa.OneOf([aa.ChangeAudioSpeed(limit=0.15, prob=0.5, sr=SR, max_duration=0.55),
                     aa.AudioDistort(limit=0.05, prob=0.5),
                     aa.PitchShift(limit=2, prob=0.5)], prob=0.9)
    ref = oaa.make_one_of([dict(kind='stretch', limit=0.15, prob=0.5, sr=SR, max_duration=0.55),
                           dict(kind='distort', limit=0.05, prob=0.5),
                           dict(kind='pitch', limit=2, prob=0.5)], 0.9)
    random.seed(5)
    np.random.seed(5)
    got = [ours(wav=aa.Wave(y), sr=SR)['wav'] for y in wavs]
    st = (random.getstate(), np.random.get_state()[1].copy())
    random.seed(5)
    np.random.seed(5)
    exp = [oaa.one_of(ref, y, SR) for y in wavs]
    assert st[0] == random.getstate() and np.array_equal(st[1], np.random.get_state()[1])
    kinds = set()
    for w, e in zip(got, exp):
        assert w.length == e.shape[0]
        kinds.update(r[0] for r in w.records)
    assert {aa.STRETCH, aa.PITCH} <= kinds


# ------------------------------------------------------------------------- device vs oracle
def _cmp(got, exp, tol):
    scale = max(np.abs(exp).max(), 1e-30)
    return np.abs(got - exp).max() / scale


@pytest.mark.gpu
def test_time_stretch_device_matches_oracle(dev):
    """Ragged batch, rates over ChangeAudioSpeed's range: device vs restatement.  librosa's
    chain carries float32 phase noise: the vocoder's float32 accumulator reaches ~1e4-1e5 rad
    in the high bins (an ulp of 1e-3-1e-2 rad), so the restatement itself sits 1e-5 (513
    samples) to 2e-2 (10 s) of the peak away from the same chain in float64
    (le.time_stretch_f64), and any last-bit difference upstream decorrelates those roundings
    (two windows 2.2e-16 apart move the restatement by 7e-5 of the peak on 1 s;
    scripts/diag_stretch.py).  The device's fp64 radix-2 FFTs differ from pocketfft in those
    last bits, so the bound is relative to that noise: the device is closer to the
    restatement than 3/4 of the restatement's own distance from float64, and no farther from
    float64 than 1.5x the restatement."""
    lens = [16000, 9001, 23456, 4096, 513, 160000]
    rates = [0.85, 1.15, 0.93, 1.0, 1.07, 0.891]
    wavs = [_speech_like(n, i) for i, n in enumerate(lens)]
    pcm = torch.zeros(len(wavs), max(lens))
    for i, y in enumerate(wavs):
        pcm[i, :len(y)] = torch.from_numpy(y)
    out, olens = ops.time_stretch(pcm.to(dev), lens, rates)
    out = out.cpu().numpy()
    for i, (y, r) in enumerate(zip(wavs, rates)):
        e = le.time_stretch(y, r)
        f = le.time_stretch_f64(y, r)
        assert olens[i] == len(e)
        noise = _cmp(e, f, 0)
        err = _cmp(out[i, :len(e)], e, 0)
        err64 = _cmp(out[i, :len(e)], f, 0)
        assert err <= 0.75 * noise + 2e-6, (i, r, err, noise)
        assert err64 <= 1.5 * noise + 2e-6, (i, r, err64, noise)
        assert not out[i, len(e):].any()


@pytest.mark.gpu
@pytest.mark.parametrize("pairs", [[(16000, 8000), (8000, 16000), (22050, 16000)],
                                   [(44100, 16000), (16000, 17959.5), (16000 / 0.891, 16000)]])
def test_resample_device_matches_oracle(dev, pairs):
    """resampy kaiser_best on the device vs the restatement (same tap order, fp64 products
    and sums without contraction, float32 accumulation): within 2 float32 ulps."""
    lens = [12345, 30000, 777][:len(pairs)]
    wavs = [_speech_like(n, 10 + i) for i, n in enumerate(lens)]
    pcm = torch.zeros(len(wavs), max(lens))
    for i, y in enumerate(wavs):
        pcm[i, :len(y)] = torch.from_numpy(y)
    ratios = [float(b) / a for a, b in pairs]
    out, olens = ops.resample(pcm.to(dev), lens, ratios)
    out = out.cpu().numpy()
    for i, (y, (a, b)) in enumerate(zip(wavs, pairs)):
        e = le.resampy_resample(y, a, b)
        assert olens[i] == len(e)
        d = np.abs(out[i, :len(e)] - e)
        assert (d <= 2 * np.spacing(np.abs(e).astype(np.float32)) + 1e-12).all(), (i, d.max())


@pytest.mark.gpu
def test_pitch_shift_and_file_resample_through_apply_waves(dev):
    """Records (a file at 22.05 kHz resampled at load, then PitchShift / ChangeAudioSpeed /
    AudioDistort) replayed by apply_waves vs the oracle's librosa chain."""
    specs = [('pitch', 1.3), ('stretch', 1.1), ('pitch', -2.0), ('none', 0), ('distort', 0)]
    waves, exp = [], []
    for i, (kind, v) in enumerate(specs):
        y = _speech_like(9000 + 1000 * i, 20 + i)
        w = aa.Wave(y)
        e = y
        if i % 2 == 0:           # a 22.05 kHz file
            w.record(aa.RESAMPLE, a=22050, b=SR)
            w.length = aa.heavy_length(aa.RESAMPLE, 22050, SR, 0.0, w.length)
            e = le.resample(e, 22050, SR)
        if kind == 'pitch':
            w.record(aa.PITCH, a=SR, alpha=v)
            e = le.pitch_shift(e, SR, v)
        elif kind == 'stretch':
            w.record(aa.STRETCH, alpha=v)
            w.length = ops.stretch_plan(w.length, v)[0]
            e = le.time_stretch(e, v)
        elif kind == 'distort':
            w.record(aa.DISTORT, alpha=float(np.float32(1.02)))
            e = np.clip(np.float32(1.02) * e, 0, e.max()).astype(np.float32)
        waves.append(w)
        exp.append(e)
    out, lens = aa.apply_waves(waves, dev)
    out = out.cpu().numpy()
    for i, e in enumerate(exp):
        assert lens[i] == len(e)
        # the phase-vocoder bound of test_time_stretch_device_matches_oracle (pitch shift is
        # a stretch plus a resample; the float32 phase noise of these <= 1 s signals is
        # 1e-5-1e-3 of the peak)
        assert _cmp(out[i, :len(e)], e, 0) < 5e-4, i
        assert not out[i, len(e):].any()


@pytest.mark.gpu
def test_parse_audio_full_aug_type0_pipeline(dev, tmp_path):
    """SpectrogramParser.parse_audio with the reference's full aug_type-0 OneOf (AddNoise,
    ChangeAudioSpeed, AudioDistort, Shift, PitchShift; data_loader_aug.py:369-388): device
    augmentation + STFT against the oracle spectrogram of the oracle-augmented waveform."""
    from scipy.io import wavfile
    from ds2amd.data_loader import SpectrogramParser
    rng = np.random.default_rng(3)
    nz = str(tmp_path / "noise.wav")
    wavfile.write(nz, SR, (rng.standard_normal(60000) * 3000).astype(np.int16))
    paths = []
    for i in range(10):
        p = str(tmp_path / f"u{i}.wav")
        wavfile.write(p, SR, (_speech_like(int(rng.integers(8000, 20000)), 40 + i) * 20000)
                      .astype(np.int16))
        paths.append(p)
    conf = dict(sample_rate=SR, window_size=0.02, window_stride=0.01, window='hamming',
                noise_prob=0.7, noise_dir=str(tmp_path / "noise*.wav"))
    parser = SpectrogramParser(conf, normalize='max_frame', augment=False, device=dev)
    ref = oaa.make_one_of([dict(kind='noise', limit=0.2, prob=0.7, noise_samples=[nz]),
                           dict(kind='stretch', limit=0.15, prob=0.7, sr=SR, max_duration=10),
                           dict(kind='distort', limit=0.05, prob=0.7),
                           dict(kind='shift', limit=SR * 0.5, prob=0.7, sr=SR, max_duration=10),
                           dict(kind='pitch', limit=2, prob=0.7)], 0.7)
    seen = set()
    for i, p in enumerate(paths):
        random.seed(100 + i)
        np.random.seed(100 + i)
        got = parser.parse_audio(p).cpu()
        random.seed(100 + i)
        np.random.seed(100 + i)
        np.random.uniform(0.85, 1.15)
        np.random.uniform(-10, 10)
        y, _ = oaa._read_norm(p)
        y = oaa.one_of(ref, y, SR)
        exp = orc.spectrogram(y)
        assert got.shape == exp.shape
        # the noise scale of librosa's float32 phase vocoder on this utterance: the same draws
        # through the float64 chain (test_time_stretch_device_matches_oracle)
        random.seed(100 + i)
        np.random.seed(100 + i)
        np.random.uniform(0.85, 1.15)
        np.random.uniform(-10, 10)
        ts = le.time_stretch
        le.time_stretch = lambda w, r: le.time_stretch_f64(w, r).astype(np.float32)
        try:
            y64 = oaa.one_of(ref, oaa._read_norm(p)[0], SR)
        finally:
            le.time_stretch = ts
        noise = (exp - orc.spectrogram(y64)).abs().max().item()
        assert (got - exp).abs().max().item() <= 0.75 * noise + 2e-3, (i, noise)
        seen.update(t['kind'] for t in ref['transforms'] if t['prob'] == 1.0)
    assert {'stretch', 'pitch'} <= seen
