"""Spectrogram augmentations of the reference's training loader, device-applied.

ref data/spectrogram_aug.py:19-117 (SOneOf, FrequencyMask, TimeMask) wired at
data/data_loader_aug.py:421-433 and applied at :241-248 together with the
`aug_prob_8khz` cut, on |STFT| before the log / 'max_frame' normalisation.

The random draws stay on the host and follow the reference's calls on Python's
`random` module one for one (including SOneOf setting the chosen transform's `prob`
to 1 for good, a side effect of the reference), so a seeded run draws the same bands.
Instead of zeroing a numpy spectrogram, every transform returns the bands it would
zero; `SpectAugmenter.masks` packs them into the int32 [N, 9] rows that
`ds2_stft_logmag_masked` applies inside the STFT kernel.
"""
from __future__ import annotations

import random as _random
from typing import List, Optional, Sequence, Tuple

import torch

Band = Tuple[int, int]


class FrequencyMask:
    """ref spectrogram_aug.py:64-84."""
    kind = "freq"

    def __init__(self, bands=2, prob=.25, dropout_width=10):
        assert dropout_width > 0
        self.bands = bands
        self.prob = prob
        self.dropout_width = dropout_width

    def draw(self, freqs: int, frames: int, rng=_random) -> List[Band]:
        assert self.dropout_width < freqs
        out = []
        for _ in range(self.bands):
            if rng.random() < self.prob:
                band_width = rng.randint(0, int(self.dropout_width))
                band_center = rng.randint(0, freqs)
                lower = max(0, int(band_center - band_width // 2))
                higher = min(int(band_center + band_width // 2), freqs)
                out.append((lower, higher))
        return out


class TimeMask:
    """ref spectrogram_aug.py:87-117."""
    kind = "time"

    def __init__(self, bands=2, prob=.25, dropout_length=50, max_dropout_ratio=.15):
        assert dropout_length > 0
        self.bands = bands
        self.prob = prob
        self.dropout_length = dropout_length
        self.max_dropout_ratio = max_dropout_ratio

    def draw(self, freqs: int, frames: int, rng=_random) -> List[Band]:
        out = []
        for _ in range(self.bands):
            if rng.random() < self.prob:
                band_width = rng.randint(0, int(self.dropout_length))
                band_width = min(band_width, int(self.max_dropout_ratio * frames))
                band_center = rng.randint(0, frames)
                lower = max(0, int(band_center - band_width // 2))
                higher = min(int(band_center + band_width // 2), frames)
                out.append((lower, higher))
        return out


class SOneOf:
    """ref spectrogram_aug.py:19-29: with probability `prob` one transform, chosen
    uniformly, runs with its prob set to 1 (permanently, as in the reference)."""

    def __init__(self, transforms, prob=0.5):
        self.transforms = transforms
        self.prob = prob

    def draw(self, freqs: int, frames: int, rng=_random):
        if rng.random() < self.prob:
            t = rng.choice(self.transforms)
            t.prob = 1.
            return t.kind, t.draw(freqs, frames, rng)
        return None, []


class SpectAugmenter:
    """The loader's spectrogram augmentation state (data_loader_aug.py:357-359,421-433):
    `noise_prob` (the SOneOf probability), `aug_prob_spect`, `aug_prob_8khz`."""

    def __init__(self, audio_conf, rng=None):
        self.rng = rng if rng is not None else _random
        self.aug_prob = audio_conf.get('noise_prob') or 0
        self.aug_prob_spect = audio_conf.get('aug_prob_spect') or 0
        self.aug_prob_8khz = audio_conf.get('aug_prob_8khz') or 0
        self.augs_spect = None
        if self.aug_prob_spect > 0:
            self.augs_spect = SOneOf([
                FrequencyMask(bands=2, prob=self.aug_prob_spect, dropout_width=20),
                TimeMask(bands=2, prob=self.aug_prob_spect, dropout_length=50,
                         max_dropout_ratio=.15)], prob=self.aug_prob)

    @property
    def active(self) -> bool:
        return self.augs_spect is not None or self.aug_prob_8khz > 0

    def draw_one(self, freqs: int, frames: int) -> List[int]:
        """One utterance's mask row {f_lo0, f_hi0, f_lo1, f_hi1, t_lo0, t_hi0, t_lo1,
        t_hi1, f_cut}, drawing in the reference's order (augs_spect, then the 8 kHz cut)."""
        row = [0, 0, 0, 0, 0, 0, 0, 0, freqs]
        if self.augs_spect is not None:
            kind, bands = self.augs_spect.draw(freqs, frames, self.rng)
            base = 0 if kind == "freq" else 4
            for i, (lo, hi) in enumerate(bands[:2]):
                row[base + 2 * i] = lo
                row[base + 2 * i + 1] = hi
        if self.aug_prob_8khz > 0:
            if self.rng.random() < self.aug_prob_8khz:
                row[8] = min(81, freqs)        # spect[81:] = 0
        return row

    def masks(self, freqs: int, frames: Sequence[int], device) -> Optional[torch.Tensor]:
        if not self.active:
            return None
        rows = [self.draw_one(freqs, int(t)) for t in frames]
        return torch.tensor(rows, dtype=torch.int32).to(device)


def apply_masks_np(spect, row):
    """CPU application of one mask row to a magnitude spectrogram [F, T] (in place);
    the reference's `spect[lo:hi, :] = 0` / `spect[:, lo:hi] = 0` / `spect[81:] = 0`."""
    for i in range(2):
        lo, hi = row[2 * i], row[2 * i + 1]
        spect[lo:hi, :] = 0
        lo, hi = row[4 + 2 * i], row[4 + 2 * i + 1]
        spect[:, lo:hi] = 0
    spect[row[8]:] = 0
    return spect
