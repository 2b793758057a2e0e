"""Waveform augmentations (data/audio_aug.py): host draws vs the oracle restatement on
CPU, the device replay (ds2_wave_aug) vs the oracle's numpy arithmetic on the GPU, and
the augmented front-end end to end (SpectrogramParser.parse_audio)."""
import copy
import random

import numpy as np
import pytest
import torch

from ds2amd import audio_aug as aa
from oracle import audio_aug as oaa
from oracle import ds2_oracle as orc

SR = 16000


def _noise_file(tmp_path, n=20000, seed=1):
    from scipy.io import wavfile
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(n) * 3000).astype(np.int16)
    path = str(tmp_path / "noise.wav")
    wavfile.write(path, SR, x)
    return path


def _utterances(k=40, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(k):
        y = rng.standard_normal(int(rng.integers(2000, 9000))).astype(np.float32)
        out.append(y / np.abs(y).max())
    return out


def _pipelines(noise_path, prob=0.5, p=0.8):
    ours = aa.OneOf([aa.AddNoise(limit=0.2, prob=prob, noise_samples=[noise_path]),
                     aa.AudioDistort(limit=0.05, prob=prob),
                     aa.Shift(limit=SR * 0.05, prob=prob, sr=SR, max_duration=0.6)], prob=p)
    ref = oaa.make_one_of([
        dict(kind='noise', limit=0.2, prob=prob, noise_samples=[noise_path]),
        dict(kind='distort', limit=0.05, prob=prob),
        dict(kind='shift', limit=SR * 0.05, prob=prob, sr=SR, max_duration=0.6)], p)
    return ours, ref


def _replay(w: aa.Wave) -> np.ndarray:
    """numpy replay of a Wave's records with the kernel's stated semantics (fp32 between
    ops, float64 noise mix) -- checks the records on the host."""
    y = w.samples.astype(np.float32)
    for kind, a, b, alpha, nz in w.records:
        if kind == aa.SHIFT:
            z = np.zeros(y.shape[0] + b, np.float32)
            z[a:a + y.shape[0]] = y
            y = z
        elif kind == aa.DISTORT:
            y = np.clip(np.float32(alpha) * y, 0, y.max()).astype(np.float32)
        else:
            y = ((y.astype(np.float64) + alpha * nz) / (1 + alpha)).astype(np.float32)
    return y


def _run_both(noise_path, wavs, seed=123):
    ours, ref = _pipelines(noise_path)
    random.seed(seed)
    np.random.seed(seed)
    got = [ours(wav=aa.Wave(y), sr=SR)['wav'] for y in wavs]
    st_ours = (random.getstate(), np.random.get_state()[1].copy())
    random.seed(seed)
    np.random.seed(seed)
    exp = [oaa.one_of(ref, y, SR) for y in wavs]
    st_ref = (random.getstate(), np.random.get_state()[1].copy())
    return got, exp, st_ours, st_ref


def test_draws_and_records_match_oracle(tmp_path):
    """Same `random` / `np.random` sequence as the restated reference (final RNG states
    equal), same lengths, and the records replayed in numpy equal the oracle's output."""
    wavs = _utterances()
    got, exp, st_ours, st_ref = _run_both(_noise_file(tmp_path), wavs)
    assert st_ours[0] == st_ref[0]
    assert np.array_equal(st_ours[1], st_ref[1])
    kinds = set()
    for w, e in zip(got, exp):
        assert w.length == e.shape[0]
        kinds.update(r[0] for r in w.records)
        np.testing.assert_allclose(_replay(w), e, rtol=2e-7, atol=1e-7)
    assert kinds == {aa.SHIFT, aa.DISTORT, aa.NOISE}      # every op kind was exercised


def test_distort_hand_case():
    """limit 0 -> alpha 1: clip(wav, 0, max(wav)) zeroes the negative half (audio_aug.py:59,177)."""
    w = aa.AudioDistort(limit=0.0, prob=1.0)(wav=np.array([-.5, .25, 1.0], np.float32))['wav']
    assert _replay(w).tolist() == [0.0, 0.25, 1.0]


def test_librosa_transforms_record_when_drawn():
    """ChangeAudioSpeed / PitchShift record their effect (replayed by ds2_time_stretch /
    ds2_resample, tests/test_librosa_effects.py) only when their draw fires."""
    random.seed(0)
    t = aa.ChangeAudioSpeed(prob=0.0)
    w = t(wav=np.zeros(1000, np.float32))['wav']
    assert w.length == 1000 and not w.records
    w = aa.ChangeAudioSpeed(limit=0.15, prob=1.0, sr=SR, max_duration=10)(
        wav=np.zeros(1000, np.float32))['wav']
    assert w.records[0][0] == aa.STRETCH and w.length == int(round(1000 / w.records[0][3]))
    w = aa.PitchShift(prob=1.0)(wav=np.zeros(1000, np.float32), sr=SR)['wav']
    assert w.records[0][0] == aa.PITCH and w.length == 1000 and w.records[0][1] == SR


@pytest.mark.gpu
def test_wave_aug_device_matches_oracle(dev, tmp_path):
    wavs = _utterances(24, seed=3)
    got, exp, _, _ = _run_both(_noise_file(tmp_path), wavs, seed=7)
    out, lens = aa.apply_waves(got, dev)
    out = out.cpu().numpy()
    for i, e in enumerate(exp):
        assert lens[i] == e.shape[0]
        np.testing.assert_allclose(out[i, :lens[i]], e, rtol=2e-7, atol=1e-7)
        assert not out[i, lens[i]:].any()


@pytest.mark.gpu
def test_parse_audio_with_augs_matches_oracle(dev, tmp_path):
    """SpectrogramParser.parse_audio with noise_prob set: the reference's draws (tempo
    class, two sox draws, OneOf), device augmentation, device STFT -- against the oracle
    spectrogram of the oracle-augmented float64 waveform."""
    from scipy.io import wavfile
    from ds2amd.data_loader import SpectrogramParser
    noise = _noise_file(tmp_path, n=40000, seed=4)
    rng = np.random.default_rng(9)
    paths = []
    for i in range(6):
        p = str(tmp_path / f"u{i}.wav")
        wavfile.write(p, SR, (rng.standard_normal(int(rng.integers(6000, 16000))) * 4000).astype(np.int16))
        paths.append(p)
    conf = dict(sample_rate=SR, window_size=0.02, window_stride=0.01, window='hamming',
                noise_prob=0.6, noise_dir=str(tmp_path / "noise*.wav"))
    parser = SpectrogramParser(conf, normalize='max_frame', augment=False, device=dev)
    # the parser's OneOf uses the reference's aug_type-0 list; librosa-backed members are
    # replaced so every draw lands on a built transform (same list order and probs)
    parser.augs.transforms[1] = aa.AudioDistort(limit=0.05, prob=0.6)
    parser.augs.transforms[4] = aa.Shift(limit=SR * 0.5, prob=0.6, sr=SR, max_duration=10)
    ref = oaa.make_one_of([dict(kind='noise', limit=0.2, prob=0.6, noise_samples=[noise]),
                           dict(kind='distort', limit=0.05, prob=0.6),
                           dict(kind='distort', limit=0.05, prob=0.6),
                           dict(kind='shift', limit=SR * 0.5, prob=0.6, sr=SR, max_duration=10),
                           dict(kind='shift', limit=SR * 0.5, prob=0.6, sr=SR, max_duration=10)], 0.6)
    for i, p in enumerate(paths):
        random.seed(i)
        np.random.seed(i)
        got = parser.parse_audio(p).cpu()
        random.seed(i)
        np.random.seed(i)
        np.random.uniform(0.85, 1.15)
        np.random.uniform(-10, 10)
        y, _ = oaa._read_norm(p)
        y = oaa.one_of(ref, y, SR)
        exp = orc.spectrogram(y)
        assert got.shape == exp.shape
        assert (got - exp).abs().max().item() < 2e-4
