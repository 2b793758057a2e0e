"""Waveform augmentations — drop-in for the reference ``data/audio_aug.py`` on the
device front-end.

The transforms keep the reference's class names, constructor arguments, call
signature (``t(wav=..., sr=...) -> {'wav': ..., 'sr': ...}``) and — the part that
decides which augmentation an utterance gets — its exact sequence of ``random`` /
``np.random`` draws.  What they do not do is touch the samples: each one appends a
record to the :class:`Wave` it is handed, and :func:`apply_waves` replays the
records of a whole batch in one HIP launch (``ds2_wave_aug``) straight into the
device PCM buffer the STFT kernel reads.

* ``Shift`` (audio_aug.py:26-44), ``AudioDistort`` (:47-60, ``clip`` :177-178),
  ``AddNoise`` (:78-107, incl. ``get_stacked_noise`` :110-134): built.
* ``ChangeAudioSpeed`` (:7-23, librosa.effects.time_stretch) and ``PitchShift``
  (:63-75, librosa.effects.pitch_shift = time stretch + resampy resampling): their draws
  are made in the reference order and replayed on the device by ``ds2_time_stretch`` /
  ``ds2_resample`` (csrc/effects.hip, restated from librosa 0.8 / resampy 0.2; parity with
  librosa itself unpinned, it is absent here — oracle/librosa_effects.py is the checker).
  A file at another sample rate is resampled the same way (data_loader_aug.py:668).
* ``Compose`` / ``OneOf`` / ``OneOrOther`` (:137-174): same semantics, including
  ``OneOf`` setting the chosen transform's ``prob`` to 1 for good (:160).
"""
from __future__ import annotations

import random
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import ops

SHIFT, DISTORT, NOISE = 1, 2, 3          # replayed by ds2_wave_aug
STRETCH, PITCH, RESAMPLE = 4, 5, 6       # ds2_time_stretch / ds2_resample (before the above)
HEAVY = (STRETCH, PITCH, RESAMPLE)
MAX_DURATION_AUG = 10          # seconds (data_loader_aug.py:49)


class Wave(object):
    """An utterance on its way through the transforms: the loaded fp32 samples plus
    the records of what the transforms decided.  ``shape`` follows the length the
    reference's array would have, so the transforms' length checks read the same."""

    def __init__(self, samples):
        self.samples = np.ascontiguousarray(np.asarray(samples, dtype=np.float32).reshape(-1))
        self.length = int(self.samples.shape[0])
        self.records = []      # (kind, a, b, alpha, noise float64 slice or None)

    @property
    def shape(self):
        return (self.length,)

    def record(self, kind, a=0, b=0, alpha=0.0, noise=None):
        self.records.append((kind, int(a), int(b), float(alpha), noise))


def _as_wave(wav) -> Wave:
    return wav if isinstance(wav, Wave) else Wave(wav)


class ChangeAudioSpeed:
    def __init__(self, limit=0.15, prob=0.5, max_duration=10, sr=16000):
        self.limit = limit
        self.prob = prob
        self.max_duration = max_duration * sr

    def __call__(self, wav=None, sr=None):
        wav = _as_wave(wav)
        assert len(wav.shape) == 1
        if random.random() < self.prob:
            alpha = 1.0 + self.limit * random.uniform(-1, 1)
            new_len = ops.stretch_plan(wav.length, alpha)[0]     # len(time_stretch(wav, alpha))
            if new_len < self.max_duration:
                wav.record(STRETCH, alpha=alpha)
                wav.length = new_len
        return {'wav': wav, 'sr': sr}


class Shift:
    def __init__(self, limit=512, prob=0.5, max_duration=10, sr=16000):
        self.limit = int(limit)
        self.prob = prob
        self.max_duration = max_duration * sr

    def __call__(self, wav=None, sr=None):
        wav = _as_wave(wav)
        assert len(wav.shape) == 1
        if random.random() < self.prob:
            limit = self.limit
            shift = round(random.uniform(0, limit))
            if wav.length + limit < self.max_duration:
                wav.record(SHIFT, shift, limit)
                wav.length += limit
        return {'wav': wav, 'sr': sr}


class AudioDistort:
    def __init__(self, limit=0.3, prob=0.5):
        self.limit = limit
        self.prob = prob

    def __call__(self, wav=None, sr=None):
        wav = _as_wave(wav)
        if random.random() < self.prob:
            alpha = 1.0 + self.limit * random.uniform(-1, 1)
            # float32 numpy math in the reference: f32(alpha) * wav, clipped to [0, max(wav)]
            wav.record(DISTORT, alpha=float(np.float32(alpha)))
        return {'wav': wav, 'sr': sr}


class PitchShift:
    def __init__(self, limit=5, prob=0.5):
        self.limit = abs(limit)
        self.prob = prob

    def __call__(self, wav=None, sr=22050):
        wav = _as_wave(wav)
        assert len(wav.shape) == 1
        if random.random() < self.prob:
            alpha = self.limit * random.uniform(-1, 1)
            wav.record(PITCH, a=int(sr), alpha=alpha)     # length unchanged (fix_length)
        return {'wav': wav, 'sr': sr}


def get_stacked_noise(noise_path=None, wav=None, sr=16000):
    """audio_aug.py:110-134.  The reference reads one noise file; when it is shorter than
    the utterance its next iteration np.stack-s two 1-D arrays and fails its own
    ``assert len(noise.shape)==1`` — restated as that AssertionError."""
    from .data_loader import load_audio_norm
    noise, sample_rate = load_audio_norm(noise_path)
    assert len(noise.shape) == 1
    if sample_rate != sr:
        # the reference's branch resamples an undefined `y` (audio_aug.py:117-118)
        raise NameError("get_stacked_noise: name 'y' is not defined (reference "
                        "data/audio_aug.py:118 resamples an undefined variable)")
    if noise.shape[0] > wav.shape[0]:
        return noise
    assert False, "get_stacked_noise: noise shorter than the utterance (reference :123-128)"


class AddNoise:
    def __init__(self, limit=0.2, prob=0.5, noise_samples=[]):
        self.limit = abs(limit)
        self.prob = prob
        self.noise_samples = noise_samples

    def __call__(self, wav=None, sr=None):
        wav = _as_wave(wav)
        assert len(wav.shape) == 1
        for i in range(0, 2):
            if random.random() < self.prob:
                if i == 0:
                    _noise = get_stacked_noise(noise_path=random.sample(self.noise_samples, k=1)[0],
                                               wav=wav, sr=sr)
                    if _noise.shape[0] < wav.shape[0]:
                        return {'wav': wav, 'sr': sr}
                else:
                    _noise = np.random.normal(0, 1, wav.shape[0] * 2)
                alpha = self.limit * random.uniform(0, 1)
                pos = random.randint(0, _noise.shape[0] - wav.shape[0])
                seg = np.ascontiguousarray(_noise[pos:pos + wav.shape[0]], dtype=np.float64)
                wav.record(NOISE, alpha=alpha, noise=seg)
        return {'wav': wav, 'sr': sr}


class Compose(object):
    def __init__(self, transforms, p=1.):
        self.transforms = [t for t in transforms if t is not None]
        self.p = p

    def __call__(self, **data):
        if np.random.random() < self.p:
            for t in self.transforms:
                data = t(**data)
        return data


class OneOf(object):
    def __init__(self, transforms, prob=.5):
        self.transforms = transforms
        self.p = prob
        transforms_ps = [t.prob for t in transforms]
        s = sum(transforms_ps)
        self.transforms_ps = [t / s for t in transforms_ps]

    def __call__(self, **data):
        if np.random.random() < self.p:
            t = np.random.choice(self.transforms, p=self.transforms_ps)
            t.prob = 1.
            data = t(**data)
        return data


class OneOrOther(object):
    def __init__(self, first, second, prob=.5):
        self.first = first
        first.prob = 1.
        self.second = second
        second.pprob = 1.     # sic (audio_aug.py:170): the second transform keeps its prob
        self.p = prob

    def __call__(self, **data):
        return self.first(**data) if np.random.random() < self.p else self.second(**data)


def build_audio_augs(audio_conf, noise_samples: Sequence[str] = (), max_duration=None):
    """The aug_type 0 pipeline of SpectrogramDataset (data_loader_aug.py:355-418):
    OneOf([AddNoise, ChangeAudioSpeed, AudioDistort, Shift, PitchShift]) at
    ``noise_prob``; None when noise_prob <= 0."""
    aug_prob = audio_conf.get('noise_prob') or 0
    if aug_prob <= 0:
        return None
    sr = audio_conf.get('sample_rate')
    md = max_duration if max_duration is not None else MAX_DURATION_AUG
    return OneOf([
        AddNoise(limit=0.2, prob=aug_prob, noise_samples=list(noise_samples)),
        ChangeAudioSpeed(limit=0.15, prob=aug_prob, sr=sr, max_duration=md),
        AudioDistort(limit=0.05, prob=aug_prob),
        Shift(limit=sr * 0.5, prob=aug_prob, sr=sr, max_duration=md),
        PitchShift(limit=2, prob=aug_prob),
    ], prob=aug_prob)


def _heavy(kind, a, b, alpha, lens, pcm):
    """One device effect over the selected rows: -> (out [k, S'], new lengths)."""
    if kind == STRETCH:
        return ops.time_stretch(pcm, lens, alpha)
    if kind == RESAMPLE:
        ratios = [float(bb) / aa for aa, bb in zip(a, b)]                # sr_new / sr_orig
        out_lens = [int(np.ceil(l * r)) for l, r in zip(lens, ratios)]   # librosa fix_length
        return ops.resample(pcm, lens, ratios, out_lens)
    # PITCH: time_stretch by rate = 2 ** (-n / 12), resample sr / rate -> sr, fix_length(len)
    rates = [2.0 ** (-float(n) / 12) for n in alpha]
    y, ylens = ops.time_stretch(pcm, lens, rates)
    ratios = [float(sr) / (float(sr) / r) for sr, r in zip(a, rates)]
    return ops.resample(y, ylens, ratios, [int(l) for l in lens])


def heavy_length(kind, a, b, alpha, length):
    if kind == STRETCH:
        return ops.stretch_plan(length, alpha)[0]
    if kind == RESAMPLE:
        return int(np.ceil(length * (float(b) / a)))
    return length


def apply_waves(waves: Sequence[Wave], device) -> tuple:
    """Replay the records of a batch on the device: -> (pcm [N, S_max] fp32 device,
    lengths list).  The librosa effects (resample, time stretch, pitch shift) lead an
    utterance's records (a file's resampling at load, then OneOf's one transform); each
    round of them is one ds2_resample / ds2_time_stretch launch over the utterances that
    have one; the remaining records are one ds2_wave_aug launch.  Uploaded once."""
    waves = [_as_wave(w) for w in waves]
    n = len(waves)
    heavy, light = [], []
    for b, w in enumerate(waves):
        k = 0
        while k < len(w.records) and w.records[k][0] in HEAVY:
            k += 1
        if any(r[0] in HEAVY for r in w.records[k:]):
            raise NotImplementedError(f"utterance {b}: a librosa effect after a replayed "
                                      "transform (the reference's pipelines never do this)")
        heavy.append(w.records[:k])
        light.append(w.records[k:])
    s_in = max(w.samples.shape[0] for w in waves)
    pcm = np.zeros((n, max(s_in, 1)), dtype=np.float32)
    for b, w in enumerate(waves):
        pcm[b, :w.samples.shape[0]] = w.samples
    pcm_d = torch.from_numpy(pcm).to(device)
    base = [w.samples.shape[0] for w in waves]
    for h in range(max((len(r) for r in heavy), default=0)):
        outs = {}
        for kind in HEAVY:
            rows = [b for b in range(n) if len(heavy[b]) > h and heavy[b][h][0] == kind]
            if not rows:
                continue
            recs = [heavy[b][h] for b in rows]
            y, ylens = _heavy(kind, [r[1] for r in recs], [r[2] for r in recs],
                              [r[3] for r in recs], [base[b] for b in rows],
                              pcm_d[torch.tensor(rows, device=device)])
            for i, b in enumerate(rows):
                outs[b] = (y[i], ylens[i])
        new_base = [outs[b][1] if b in outs else base[b] for b in range(n)]
        nxt = torch.zeros(n, max(1, max(new_base)), device=device, dtype=torch.float32)
        for b in range(n):
            if b in outs:
                nxt[b, :new_base[b]] = outs[b][0][:new_base[b]]
            else:
                nxt[b, :base[b]] = pcm_d[b, :base[b]]
        pcm_d, base = nxt, new_base
    k = max(1, max(len(r) for r in light))
    op_i = np.zeros((n, k, 4), dtype=np.int32)
    op_f = np.zeros((n, k), dtype=np.float64)
    rows: List[np.ndarray] = []
    cap = 1
    for b, w in enumerate(waves):
        ln = base[b]
        cap = max(cap, ln)
        for j, (kind, a, bb, alpha, nz) in enumerate(light[b]):
            if kind == SHIFT:
                ln += bb
            elif kind == NOISE:
                a = len(rows)
                rows.append(nz)
            op_i[b, j] = (kind, a, bb, 0)
            op_f[b, j] = alpha
            cap = max(cap, ln)
        if ln != w.length:
            raise ValueError(f"utterance {b}: records give {ln} samples, the transforms {w.length}")
    lens = [w.length for w in waves]
    if not any(light):
        return pcm_d, lens
    # the records were validated above (every length and the buffer cap follow from them,
    # as the kernel recomputes), so the kernel's consistency word is not read back: no
    # device sync per batch
    noise = None
    if rows:
        nl = max(r.shape[0] for r in rows)
        nz = np.zeros((len(rows), nl), dtype=np.float64)
        for r, seg in enumerate(rows):
            nz[r, :seg.shape[0]] = seg
        noise = torch.from_numpy(nz).to(device)
    out = ops.wave_aug(pcm_d, torch.tensor(base, dtype=torch.int32).to(device),
                       torch.from_numpy(op_i).to(device), torch.from_numpy(op_f).to(device), noise,
                       lens, max(lens), cap, check=False)
    return out, lens
