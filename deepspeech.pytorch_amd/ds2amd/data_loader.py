"""Feature front-end and batching — drop-in for the hot-path parts of the
reference ``data/data_loader.py`` / ``data/data_loader_aug.py``.

* ``SpectrogramParser.audio_to_stft`` / ``parse_audio`` run the STFT, |.|,
  log1p and 'max_frame' normalisation as one HIP pipeline (ds2_stft_logmag) on
  the GPU instead of librosa in CPU worker processes (ref
  data_loader.py:201-220,276-284; data_loader_aug.py:220-249,297-307).
* ``SpectrogramParser.parse_batch`` takes raw PCM for a whole batch and returns
  the collated, zero-padded [N, 1, 161, T_max] device tensor directly.
* ``_collate_fn``, ``BucketingSampler``, ``DistributedBucketingSampler`` and
  ``AudioDataLoader`` keep the reference's semantics (data_loader_aug.py:523-617).
"""
from __future__ import annotations

import math
import random
from glob import glob
from typing import List, Sequence

import numpy as np
import torch
from torch.utils.data import DataLoader
from torch.utils.data.sampler import Sampler

from . import ops
from .audio_aug import RESAMPLE, Wave, apply_waves, build_audio_augs, heavy_length
from .spect_aug import SpectAugmenter

# tempo classes of the reference's legacy sox path (data_loader_aug.py:108-112); only the
# draws they cause are kept (the sox branch itself is dead code there, :690-697)
TEMPOS = {
    0: ('1.0', (1.0, 1.0)),
    1: ('0.9', (0.85, 0.95)),
    2: ('1.1', (1.05, 1.15))
}


def hamming(n: int) -> np.ndarray:
    """scipy.signal.hamming(n) (sym=True): 0.54 - 0.46 cos(2 pi k / (n - 1))."""
    if n == 1:
        return np.ones(1)
    k = np.arange(n)
    return 0.54 - 0.46 * np.cos(2.0 * np.pi * k / (n - 1))


def hann(n: int) -> np.ndarray:
    if n == 1:
        return np.ones(1)
    k = np.arange(n)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / (n - 1))


windows = {'hamming': hamming, 'hann': hann}


def gaussian_taps(sigma: float, truncate: float = 4.0) -> np.ndarray:
    """The correlation weights of scipy.ndimage.gaussian_filter1d (order 0)."""
    radius = int(truncate * float(sigma) + 0.5)
    x = np.arange(-radius, radius + 1)
    phi = np.exp(-0.5 / (sigma * sigma) * x ** 2)
    phi = phi / phi.sum()
    return phi[::-1].copy()


def load_audio_norm(path, channel=-1):
    """scipy wav read + normalise by max |x| (ref data/audio_loader.py:4-27)."""
    from scipy.io import wavfile
    sample_rate, sound = wavfile.read(path)
    abs_max = np.abs(sound).max()
    sound = sound.astype('float32')
    if abs_max > 0:
        sound *= 1 / abs_max
    if len(sound.shape) > 1:
        if sound.shape[1] == 1:
            sound = sound.squeeze()
        elif channel == -1:
            sound = sound.mean(axis=1)
        else:
            sound = sound[:, channel]
    return sound, sample_rate


def load_randomly_augmented_audio(path, sample_rate=16000, tempo_range=(0.85, 1.15),
                                  gain_range=(-10, 10), channel=-1, transforms=None):
    """data_loader_aug.py:679-699 (+ augment_audio_with_augs :660-676): the tempo and gain
    draws the reference makes (and no longer uses), the normalised wav, then the
    transforms' records.  -> (audio_aug.Wave, sample_rate)."""
    np.random.uniform(low=tempo_range[0], high=tempo_range[1])
    np.random.uniform(low=gain_range[0], high=gain_range[1])
    y, sr = load_audio_norm(path, channel=channel)
    wav = Wave(y)
    if sr != sample_rate:
        # librosa.resample(y, sr, sample_rate) (data_loader_aug.py:667-668), on the device
        wav.record(RESAMPLE, a=sr, b=sample_rate)
        wav.length = heavy_length(RESAMPLE, sr, sample_rate, 0.0, wav.length)
    if transforms is not None:
        wav = transforms(**{'wav': wav, 'sr': sample_rate})['wav']
    return wav, sample_rate


class SpectrogramParser(object):
    def __init__(self, audio_conf, cache_path=None, normalize=False, augment=False, channel=-1,
                 device=None):
        self.window_stride = audio_conf['window_stride']
        self.window_size = audio_conf['window_size']
        self.sample_rate = audio_conf['sample_rate']
        self.window = windows.get(audio_conf.get('window', 'hamming'), windows['hamming'])
        self.normalize = normalize
        self.augment = augment
        self.channel = channel
        self.cache_path = cache_path
        self.device = torch.device(device) if device is not None else torch.device('cuda')
        self._cache = {}
        # spectrogram augmentations (data_loader_aug.py:241-248), drawn on the host and
        # applied inside the STFT kernel; inactive unless audio_conf enables them
        self.spect_aug = SpectAugmenter(audio_conf)
        # waveform augmentations (data_loader_aug.py:361-418, aug_type 0), drawn on the
        # host and replayed on the device (ds2_wave_aug); None unless noise_prob > 0
        noise_dir = audio_conf.get('noise_dir')
        # glob order unsorted, as the reference's (data_loader_aug.py:363): AddNoise picks a
        # file by index, so the same draws mix in the same file on the same filesystem
        self.augs = build_audio_augs(audio_conf, glob(noise_dir) if noise_dir else ())

    def _consts(self, sample_rate):
        key = sample_rate
        if key not in self._cache:
            n_fft = int(sample_rate * (self.window_size + 1e-8))
            hop = int(sample_rate * (self.window_stride + 1e-8))
            win = torch.tensor(self.window(n_fft), dtype=torch.float64, device=self.device)
            # the gaussian_filter1d of 'max_frame' (sigma 20) / 'frame' (sigma 50)
            sigma = {1: 20, 4: 50}.get(self._mode())
            taps = None if sigma is None else torch.tensor(gaussian_taps(sigma),
                                                            dtype=torch.float32, device=self.device)
            self._cache[key] = (n_fft, hop, win, taps)
        return self._cache[key]

    # normalize_audio (data_loader_aug.py:274-313; --norm, train.py:75) -> ds2_stft_logmag mode
    NORM_MODES = {'none': 0, 'max_frame': 1, 'mean': 2, 'norm': 3, 'frame': 4}

    def _mode(self):
        if not self.normalize:
            return 0
        try:
            return self.NORM_MODES[self.normalize]
        except KeyError:
            raise ValueError(f"normalize={self.normalize!r}: the reference's modes are "
                             f"{sorted(self.NORM_MODES)} (data_loader_aug.py:274-313)") from None

    def parse_batch(self, signals: Sequence, sample_rate=None):
        """Raw PCM list (numpy arrays, or audio_aug.Wave records of augmented utterances)
        -> (spect [N,1,F,T_max] on device, frames int32 [N])."""
        sr = sample_rate or self.sample_rate
        n_fft, hop, win, taps = self._consts(sr)
        if any(isinstance(s, Wave) and s.records for s in signals):
            pcm_d, lens = apply_waves(signals, self.device)
        else:
            # no transform applied anything: the plain PCM upload, no ds2_wave_aug launch
            signals = [s.samples if isinstance(s, Wave) else s for s in signals]
            lens = [len(s) for s in signals]
            max_s = max(lens)
            pcm = np.zeros((len(signals), max_s), dtype=np.float32)
            for i, s in enumerate(signals):
                pcm[i, :len(s)] = s
            pcm_d = torch.from_numpy(pcm).to(self.device)
        ns_d = torch.tensor(lens, dtype=torch.int32).to(self.device)
        frames = [1 + n // hop for n in lens]
        masks = self.spect_aug.masks(ops.SPECT_ROWS, frames, self.device)
        out = ops.stft_logmag(pcm_d, ns_d, n_fft, hop, win, self._mode(), taps, max(frames),
                              masks=masks)
        if self.augment and self.normalize == 'max_frame':
            # one U(-0.5, 0.5) offset per utterance on its valid frames (data_loader_aug.py:213-214)
            off = (torch.rand(len(signals)) - 0.5).to(self.device)
            mask = (torch.arange(max(frames), device=self.device)[None, :] <
                    torch.tensor(frames, device=self.device)[:, None]).float()
            out = out + off[:, None, None] * mask[:, None, :]
        return out.unsqueeze(1), torch.tensor(frames, dtype=torch.int32)

    def audio_to_stft(self, y, sample_rate):
        """Single utterance (PCM or audio_aug.Wave) -> normalised spectrogram [F, T]
        (device tensor)."""
        if not isinstance(y, Wave):
            y = np.asarray(y, dtype=np.float32)
        spect, _ = self.parse_batch([y], sample_rate)
        return spect[0, 0]

    def parse_audio(self, audio_path):
        """data_loader_aug.py:163-215 with the reference's draws: tempo class (augment
        only), the two unused sox draws, then the waveform augs (self.augs)."""
        tempo_id = random.randrange(3) if self.augment else 0
        y, sr = load_randomly_augmented_audio(audio_path, self.sample_rate, channel=self.channel,
                                              tempo_range=TEMPOS[tempo_id][1],
                                              transforms=self.augs)
        return self.audio_to_stft(y, sr)

    def parse_audio_for_transcription(self, audio_path):
        return self.parse_audio(audio_path)


def _collate_fn(batch):
    """Sort by length desc, zero-pad to [N,1,F,T_max] (ref data_loader_aug.py:523-548)."""
    batch = sorted(batch, key=lambda sample: sample[0].size(1), reverse=True)
    longest_sample = max(batch, key=lambda p: p[0].size(1))[0]
    freq_size = longest_sample.size(0)
    minibatch_size = len(batch)
    max_seqlength = longest_sample.size(1)
    inputs = torch.zeros(minibatch_size, 1, freq_size, max_seqlength)
    input_percentages = torch.FloatTensor(minibatch_size)
    target_sizes = torch.IntTensor(minibatch_size)
    targets = []
    filenames = []
    for x in range(minibatch_size):
        tensor, target = batch[x][0], batch[x][1]
        filenames.append(batch[x][2] if len(batch[x]) > 2 else None)
        seq_length = tensor.size(1)
        inputs[x][0].narrow(1, 0, seq_length).copy_(tensor)
        input_percentages[x] = seq_length / float(max_seqlength)
        target_sizes[x] = len(target)
        targets.extend(target)
    targets = torch.IntTensor(targets)
    return inputs, targets, filenames, input_percentages, target_sizes


class AudioDataLoader(DataLoader):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.collate_fn = _collate_fn


class BucketingSampler(Sampler):
    def __init__(self, data_source, batch_size=1):
        self.data_source = data_source
        ids = list(range(0, len(data_source)))
        self.bins = [ids[i:i + batch_size] for i in range(0, len(ids), batch_size)]

    def __iter__(self):
        for ids in self.bins:
            np.random.shuffle(ids)
            yield ids

    def __len__(self):
        return len(self.bins)

    def shuffle(self, epoch):
        np.random.shuffle(self.bins)


class DistributedBucketingSampler(Sampler):
    """Rank r takes bins[r::world], padded to an even split (ref data_loader_aug.py:582-617)."""

    def __init__(self, data_source, batch_size=1, num_replicas=None, rank=None):
        if num_replicas is None or rank is None:
            import torch.distributed as dist
            num_replicas = dist.get_world_size() if num_replicas is None else num_replicas
            rank = dist.get_rank() if rank is None else rank
        self.data_source = data_source
        self.ids = list(range(0, len(data_source)))
        self.batch_size = batch_size
        self.bins = [self.ids[i:i + batch_size] for i in range(0, len(self.ids), batch_size)]
        self.num_replicas = num_replicas
        self.rank = rank
        self.num_samples = int(math.ceil(len(self.bins) * 1.0 / self.num_replicas))
        self.total_size = self.num_samples * self.num_replicas

    def __iter__(self):
        bins = self.bins + self.bins[:(self.total_size - len(self.bins))]
        assert len(bins) == self.total_size
        return iter(bins[self.rank::self.num_replicas])

    def __len__(self):
        return self.num_samples

    def shuffle(self, epoch):
        g = torch.Generator()
        g.manual_seed(epoch)
        bin_ids = list(torch.randperm(len(self.bins), generator=g))
        self.bins = [self.bins[i] for i in bin_ids]
