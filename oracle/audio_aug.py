"""CPU restatement of the reference waveform augmentations — TEST INFRASTRUCTURE.

Restates data/audio_aug.py's Shift (:26-44), AudioDistort (:47-60, clip :177-178),
AddNoise (:78-107, get_stacked_noise :110-134), ChangeAudioSpeed (:7-23) and PitchShift
(:63-75) (on oracle/librosa_effects.py's librosa restatement) and OneOf (:149-162) on numpy arrays,
with the reference's `random` / `np.random` calls in the reference's order and its
numpy dtypes (float32 in, float64 after Shift's np.zeros or AddNoise's float64 mix,
float32 math in AudioDistort).  Transforms are plain dicts here ({'kind', 'prob', ...});
OneOf mutates the chosen one's 'prob' to 1 like the reference (:160).

Parity: UNPINNED against the reference module itself — it imports librosa at module
level (absent in this image), so it cannot be run to make fixtures; the restatement is
checked by hand-computed cases in tests/test_audio_aug.py.
"""
from __future__ import annotations

import random

import numpy as np


def _read_norm(path):
    """data/audio_loader.py:4-28 (mono, normalised by max |x|)."""
    from scipy.io import wavfile
    sr, x = wavfile.read(path)
    peak = np.abs(x).max()
    x = x.astype('float32')
    if peak > 0:
        x *= 1 / peak
    if x.ndim > 1:
        x = x.squeeze() if x.shape[1] == 1 else x.mean(axis=1)
    return x, sr


def _shift(t, wav, sr):
    if random.random() < t['prob']:
        lim = int(t['limit'])
        s = round(random.uniform(0, lim))
        y = np.zeros(wav.shape[0] + lim)
        y[s:s + wav.shape[0]] = wav
        if y.shape[0] < t['max_duration'] * t['sr']:
            wav = y
    return wav


def _distort(t, wav, sr):
    if random.random() < t['prob']:
        a = 1.0 + t['limit'] * random.uniform(-1, 1)
        wav = np.clip(a * wav, 0, np.max(wav)).astype(wav.dtype)
    return wav


def _add_noise(t, wav, sr):
    for i in (0, 1):
        if random.random() >= t['prob']:
            continue
        if i == 0:
            nz, nsr = _read_norm(random.sample(t['noise_samples'], k=1)[0])
            assert nsr == sr and nz.shape[0] > wav.shape[0]
        else:
            nz = np.random.normal(0, 1, wav.shape[0] * 2)
        a = t['limit'] * random.uniform(0, 1)
        p = random.randint(0, nz.shape[0] - wav.shape[0])
        wav = (wav + a * nz[p:p + wav.shape[0]]) / (1 + a)
    return wav


def _stretch(t, wav, sr):
    """ChangeAudioSpeed (audio_aug.py:7-23) on the librosa restatement."""
    from oracle import librosa_effects as le
    if random.random() < t['prob']:
        a = 1.0 + t['limit'] * random.uniform(-1, 1)
        y = le.time_stretch(wav, a)
        if y.shape[0] < t['max_duration'] * t['sr']:
            wav = y
    return wav


def _pitch(t, wav, sr):
    """PitchShift (audio_aug.py:63-75) on the librosa restatement."""
    from oracle import librosa_effects as le
    if random.random() < t['prob']:
        a = t['limit'] * random.uniform(-1, 1)
        wav = le.pitch_shift(wav, sr, n_steps=a)
    return wav


APPLY = {'shift': _shift, 'distort': _distort, 'noise': _add_noise, 'stretch': _stretch,
         'pitch': _pitch}


def make_one_of(transforms, p):
    """OneOf's constructor (audio_aug.py:150-155): the choice weights are the probs at
    construction time, normalised, and never recomputed."""
    w = [t['prob'] for t in transforms]
    return {'transforms': transforms, 'p': p, 'w': [x / sum(w) for x in w]}


def one_of(o, wav, sr):
    """OneOf.__call__ (audio_aug.py:157-162)."""
    if np.random.random() < o['p']:
        t = o['transforms'][np.random.choice(len(o['transforms']), p=o['w'])]
        t['prob'] = 1.
        wav = APPLY[t['kind']](t, wav, sr)
    return wav
