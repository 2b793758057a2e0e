"""CPU restatement of the reference DS2 hot path — TEST INFRASTRUCTURE (the checker).

Each function restates one piece of /root/reference (file:line cited) using the
same stock CPU operators the reference path runs on (torch conv2d / batch_norm /
GRU / ctc_loss, numpy FFT), so that the HIP path can be compared against it on
identical inputs.  Nothing in the product path imports this module.

Pinning (tests/test_oracle_golden.py):
  * model forward, per-layer activations, BN running stats, greedy decode,
    get_seq_lens and one full SGD step are pinned against golden vectors that
    tests/golden/make_golden.py produced by importing the reference's own
    model.py / decoder.py in the build container (committed .npz fixtures);
  * CTC: warpctc_pytorch is absent and unpinned here; the oracle uses
    torch.nn.functional.ctc_loss (sum reduction on log_softmax), identical in
    cost and d/dacts for feasible alignments, pinned by hand-computed small
    cases in the tests;
  * STFT: librosa is absent, so the spectrogram restatement is "parity
    unpinned" against librosa itself; it is pinned by analytic known answers
    (pure tones on exact bins, silence, DC) in the tests.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F
from torch.nn.utils.rnn import pack_padded_sequence, pad_packed_sequence

LABELS = "_'ABCDEFGHIJKLMNOPQRSTUVWXYZ2 "   # labels.json:1-31


# ----------------------------------------------------------------------------
# features: data/data_loader.py:201-220,276-284; data/data_loader_aug.py:220-249,297-307
def hamming(n: int) -> np.ndarray:
    """scipy.signal.hamming(n) (symmetric; data_loader_aug.py:52-55)."""
    k = np.arange(n)
    return 0.54 - 0.46 * np.cos(2.0 * np.pi * k / (n - 1))


def stft_magnitude(y: np.ndarray, sample_rate=16000, window_size=0.02, window_stride=0.01):
    """librosa.stft(center=True, reflect pad) |.| -> float32 [n_fft/2+1, T]."""
    n_fft = int(sample_rate * (window_size + 1e-8))
    hop = int(sample_rate * (window_stride + 1e-8))
    y = np.asarray(y, dtype=np.float32)
    yp = np.pad(y, n_fft // 2, mode='reflect')
    n_frames = 1 + (len(yp) - n_fft) // hop
    idx = np.arange(n_fft)[None, :] + hop * np.arange(n_frames)[:, None]
    frames = yp[idx].astype(np.float64) * hamming(n_fft)[None, :]
    spec = np.fft.rfft(frames, axis=1).astype(np.complex64).T   # [F, T] complex64
    return np.abs(spec)


def rows161(spect: np.ndarray) -> np.ndarray:
    """data_loader_aug.py:233-238,249 on the magnitude: fewer than 161 bins (sample rates
    below 16 kHz) -> ``spect.resize((161, T)); spect[81:] = spect[80:0:-1]``; then
    ``spect[:161]``.  librosa < 0.10 allocates the stft matrix Fortran-ordered and np.abs
    keeps that order (so does stft_magnitude above), and ndarray.resize works on the memory
    order: row r <= 80 of column t receives flat value 161 t + r of the frame-major data
    (zeros past its end), not row r of frame t.  Restated literally; parity with librosa
    itself is unpinned (absent here)."""
    shape = spect.shape
    if shape[0] < 161:
        spect = spect.copy(order='K')
        spect.resize((161, *shape[1:]), refcheck=False)
        spect[81:] = spect[80:0:-1]
    return spect[:161]


def gaussian_filter1d_reflect(x: np.ndarray, sigma: float, truncate: float = 4.0):
    """scipy.ndimage.gaussian_filter1d(x, sigma) for 1-D float32 x (mode 'reflect')."""
    from scipy.ndimage import gaussian_filter1d
    return gaussian_filter1d(x, sigma, truncate=truncate)


def normalize_max_frame(spect: np.ndarray) -> torch.Tensor:
    """normalize_audio('max_frame') (data_loader_aug.py:297-307)."""
    s = np.log1p(spect * 1048576)
    s = torch.FloatTensor(s)
    mean = s.mean(dim=0, keepdim=True)
    mean = torch.FloatTensor(gaussian_filter1d_reflect(mean.numpy(), 20))
    max_mean = mean.mean()
    s.add_(-max_mean)
    return s


def normalize_audio(spect: np.ndarray, normalize) -> torch.Tensor:
    """normalize_audio (data_loader_aug.py:274-313), every mode, same op order and dtypes:
    numpy log1p on the float32 magnitude, then float32 torch reductions."""
    if normalize == 'mean':                                   # :276-280
        s = torch.FloatTensor(np.log1p(spect))
        s.add_(-s.mean())
        return s
    if normalize == 'norm':                                   # :281-287
        s = torch.FloatTensor(np.log1p(spect))
        s.add_(-s.mean())
        std = s.std(dim=0, keepdim=True)
        s.div_(std.mean())
        return s
    if normalize == 'frame':                                  # :288-296
        s = torch.FloatTensor(np.log1p(spect))
        mean = s.mean(dim=0, keepdim=True)
        mean = torch.FloatTensor(gaussian_filter1d_reflect(mean.numpy(), 50))
        s.add_(-mean.mean())
        return s
    if normalize == 'max_frame':                              # :297-307
        return normalize_max_frame(spect)
    if not normalize or normalize == 'none':                  # :308-310
        return torch.FloatTensor(np.log1p(spect))
    raise Exception("No such normalization")                  # :311-312


def spectrogram(y, sample_rate=16000, window_size=0.02, window_stride=0.01,
                normalize='max_frame') -> torch.Tensor:
    mag = rows161(stft_magnitude(y, sample_rate, window_size, window_stride))
    return normalize_audio(mag, normalize)


# ----------------------------------------------------------------------------
# model: model.py:183-393
def get_seq_lens(lengths: torch.Tensor) -> torch.Tensor:
    """model.py:382-393 with the DS2 conv params (time axis: k 11, s 2 then s 1, p 5)."""
    seq_len = lengths
    for (k, s, p) in ((11, 2, 5), (11, 1, 5)):
        seq_len = ((seq_len + 2 * p - 1 * (k - 1) - 1) / s + 1)
    return seq_len.int()


def input_sizes_quirk(input_percentages: torch.Tensor, t_max: int) -> torch.Tensor:
    """train.py:557: input_percentages.mul_(T).int() (float32 round trip)."""
    return input_percentages.clone().mul_(int(t_max)).int()


def _mask_time(x: torch.Tensor, lens: torch.Tensor) -> torch.Tensor:
    """MaskConv mask (model.py:69-78) as a bool mask."""
    t = x.shape[-1]
    m = torch.arange(t, device=x.device)[None, :] >= lens.to(x.device)[:, None].long()
    return x.masked_fill(m[:, None, None, :], 0)


class OracleDS2:
    """Functional DS2 forward on CPU from a (reference-compatible) state_dict."""

    def __init__(self, state_dict: Dict[str, torch.Tensor], nb_layers: int, hidden: int,
                 bidirectional: bool = True, bnm: float = 0.1, rnn_type: str = 'gru'):
        self.sd = {k: v.detach().clone().float() if v.is_floating_point() else v.clone()
                   for k, v in state_dict.items()}
        self.nb_layers = nb_layers
        self.hidden = hidden
        self.bidirectional = bidirectional
        self.bnm = bnm
        self.rnn_type = rnn_type

    def parameters(self) -> Dict[str, torch.Tensor]:
        return {k: v for k, v in self.sd.items()
                if not (k.endswith('running_mean') or k.endswith('running_var')
                        or k.endswith('num_batches_tracked'))}

    def _bn(self, x, prefix, training):
        return F.batch_norm(x, self.sd[prefix + '.running_mean'], self.sd[prefix + '.running_var'],
                            self.params[prefix + '.weight'], self.params[prefix + '.bias'],
                            training=training, momentum=self.bnm, eps=1e-5)

    def conv_block(self, x: torch.Tensor, out_lens: torch.Tensor, training: bool = True,
                   acts: Optional[dict] = None) -> torch.Tensor:
        """The conv stack (model.py:208-215) with MaskConv after each module (model.py:63-79)
        and the T x N x H collapse (model.py:360-362), in the dtype of x and self.params
        (the parameters: self.params as set by forward, or the caller's)."""
        p = self.params
        x = F.conv2d(x, p['conv.seq_module.0.weight'], p['conv.seq_module.0.bias'], stride=(2, 2),
                     padding=(20, 5))
        x = _mask_time(x, out_lens)
        x = self._bn(x, 'conv.seq_module.1', training)
        x = _mask_time(x, out_lens)
        x = _mask_time(F.hardtanh(x, 0, 20), out_lens)
        if acts is not None:
            acts['conv1'] = x
        x = F.conv2d(x, p['conv.seq_module.3.weight'], p['conv.seq_module.3.bias'], stride=(2, 1),
                     padding=(10, 5))
        x = _mask_time(x, out_lens)
        x = self._bn(x, 'conv.seq_module.4', training)
        x = _mask_time(x, out_lens)
        x = _mask_time(F.hardtanh(x, 0, 20), out_lens)
        if acts is not None:
            acts['conv2'] = x
        n, c, d, t = x.shape
        return x.view(n, c * d, t).transpose(1, 2).transpose(0, 1).contiguous()   # T x N x H

    def forward(self, x: torch.Tensor, lengths: torch.Tensor, training: bool = True,
                params: Optional[Dict[str, torch.Tensor]] = None, keep: bool = False):
        """Returns (logits [N,T',C], probs, out_lens int32, acts dict)."""
        self.params = params if params is not None else self.parameters()
        p = self.params
        acts = {}
        out_lens = get_seq_lens(lengths.cpu().int())
        x = self.conv_block(x, out_lens, training, acts if keep else None)
        for i in range(self.nb_layers):
            pre = f'rnns.{i}'
            if i > 0:    # SequenceWise(BatchNorm1d) (model.py:100-101)
                tt, nn_ = x.shape[0], x.shape[1]
                x = self._bn(x.view(tt * nn_, -1), pre + '.batch_norm.module', training).view(tt, nn_, -1)
            x = self._gru(x, out_lens, pre + '.rnn')
            if keep:
                acts[f'rnn{i}'] = x
        if not self.bidirectional:   # model.py:369-371: Lookahead + Hardtanh(0, 20)
            x = F.hardtanh(lookahead(x, p['lookahead.0.weight']), 0, 20)
            if keep:
                acts['lookahead'] = x
        tt, nn_ = x.shape[0], x.shape[1]
        y = self._bn(x.reshape(tt * nn_, -1), 'fc.0.module.0', training)
        y = y @ p['fc.0.module.1.weight'].t()
        x = y.view(tt, nn_, -1).transpose(0, 1)
        probs = F.softmax(x, dim=-1)
        return x, probs, out_lens, acts

    def _gru(self, x, lens, pre):
        """pack -> nn.GRU / nn.LSTM / nn.RNN -> pad -> sum directions (model.py:97-109)."""
        p = self.params
        t = x.shape[0]
        inp = x.shape[2]
        cls = {'gru': torch.nn.GRU, 'lstm': torch.nn.LSTM, 'rnn': torch.nn.RNN}[self.rnn_type]
        gru = cls(inp, self.hidden, bidirectional=self.bidirectional, bias=True)
        names = ['weight_ih_l0', 'weight_hh_l0', 'bias_ih_l0', 'bias_hh_l0']
        if self.bidirectional:
            names += [nm + '_reverse' for nm in names]
        # functional call with the (possibly autograd-tracked) tensors
        weights = {nm: p[f'{pre}.{nm}'] for nm in names}
        packed = pack_padded_sequence(x, lens.cpu().numpy(), enforce_sorted=False)
        out, _ = torch.func.functional_call(gru, weights, (packed,))
        out, _ = pad_packed_sequence(out, total_length=t)
        if self.bidirectional:
            out = out.view(out.size(0), out.size(1), 2, -1).sum(2).view(out.size(0), out.size(1), -1)
        return out


def lookahead(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """Lookahead.forward (model.py:158-172): zero-pad `context` steps at the end, stack
    the [t, t+context] windows, weight per feature and sum.  x [T, N, H], weight [H, C+1]."""
    context = weight.shape[1] - 1
    seq_len = x.size(0)
    padded = torch.cat((x, x.new_zeros(context, *x.shape[1:])), 0)
    win = torch.stack([padded[i:i + context + 1] for i in range(seq_len)])   # T x L x N x H
    return torch.mul(win.permute(0, 2, 3, 1), weight).sum(dim=3)


# ----------------------------------------------------------------------------
# CTC (warpctc_pytorch stand-in, train.py:600-602)
def ctc_loss(acts_tnc: torch.Tensor, labels: torch.Tensor, act_lens: torch.Tensor,
             label_lens: torch.Tensor, blank: int = 0, zero_infinity: bool = False):
    """Summed CTC cost over the batch (softmax inside) and d cost / d acts."""
    a = acts_tnc.detach().clone().requires_grad_(True)
    lp = F.log_softmax(a, dim=2)
    loss = F.ctc_loss(lp, labels.long(), act_lens.long(), label_lens.long(), blank=blank,
                      reduction='sum', zero_infinity=zero_infinity)
    loss.backward()
    return loss.detach(), a.grad.detach()


def ctc_costs(acts_tnc, labels, act_lens, label_lens, blank=0):
    lp = F.log_softmax(acts_tnc.double(), dim=2)
    return F.ctc_loss(lp, labels.long(), act_lens.long(), label_lens.long(), blank=blank,
                      reduction='none', zero_infinity=False).float()


# ----------------------------------------------------------------------------
# greedy decoder: decoder.py:146-197
def greedy_decode(probs: torch.Tensor, sizes: Optional[Sequence[int]], labels: str = LABELS,
                  blank_index: int = 0):
    """Pure-Python restatement of GreedyDecoder.decode (argmax -> process_string)."""
    _, max_probs = torch.max(probs, 2)
    int_to_char = dict(enumerate(labels))
    space_index = labels.index(' ') if ' ' in labels else len(labels)
    strings, offsets = [], []
    for x in range(max_probs.shape[0]):
        seq = max_probs[x].tolist()
        size = int(sizes[x]) if sizes is not None else len(seq)
        s, off = '', []
        for i in range(size):
            ch = int_to_char[seq[i]]
            if ch != int_to_char[blank_index]:
                if i != 0 and ch == int_to_char[seq[i - 1]]:
                    pass
                elif ch == labels[space_index]:
                    s += ' '
                    off.append(i)
                else:
                    s += ch
                    off.append(i)
        strings.append([s])
        offsets.append([torch.tensor(off, dtype=torch.int)])
    return strings, offsets


# ----------------------------------------------------------------------------
# training step: train.py:555-632 (+ build_optimizer train.py:139-152)
def train_step(model: OracleDS2, x, input_percentages, targets, target_sizes, lr=3e-4,
               momentum=0.9, max_norm=100.0, momentum_buffers: Optional[dict] = None,
               plant_nan: Optional[torch.Tensor] = None):
    """One reference training step on CPU.  Returns (loss, new_params, buffers, grads, norm).

    plant_nan: optional bool mask over the logits [N, T', C] set to NaN right after the
    forward (a test hook standing in for bad data); the step then follows train.py:595-598
    (NaN logits zeroed in place, zero gradient there) and, as the reference does once
    they are zeroed, always steps (the skip at :625 cannot fire).
    """
    input_sizes = input_sizes_quirk(input_percentages, x.shape[3])
    params = {k: v.detach().clone().requires_grad_(True) for k, v in model.parameters().items()}
    logits, probs, out_lens, _ = model.forward(x, input_sizes, training=True, params=params)
    if plant_nan is not None:
        logits = logits.masked_fill(plant_nan, float('nan'))
    acts = logits.transpose(0, 1)
    if torch.isnan(acts).any():                   # train.py:595-598
        acts = acts.clone()
        acts[torch.isnan(acts)] = 0
    lp = F.log_softmax(acts, dim=2)
    loss = F.ctc_loss(lp, targets.long().to(lp.device), out_lens.long(), target_sizes.long(),
                      blank=0, reduction='sum') / x.shape[0]
    loss.backward()
    grads = {k: v.grad.detach().clone() for k, v in params.items()}
    # clip_grad_norm_ (train.py:622-623)
    total = torch.norm(torch.stack([torch.norm(g, 2.0) for g in grads.values()]), 2.0)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0) if max_norm > 0 else torch.tensor(1.0)
    bufs = {} if momentum_buffers is None else dict(momentum_buffers)
    new = {}
    for k, g in grads.items():
        g = g * coef
        b = bufs.get(k)
        b = g.clone() if b is None else b * momentum + g
        bufs[k] = b
        d = g + momentum * b                      # nesterov
        new[k] = params[k].detach() - lr * d
    return loss.detach(), new, bufs, grads, total.detach()


def momentum_from_optim_dict(param_names: Sequence[str], optim_dict: dict) -> dict:
    """torch.optim.SGD state_dict (model.py:446 package['optim_dict']) -> {name: momentum
    buffer}; the SGD's params are model.parameters() in registration order (train.py:939)."""
    group = optim_dict['param_groups'][0]
    out = {}
    for name, idx in zip(param_names, group['params']):
        st = optim_dict['state'].get(idx)
        if st and st.get('momentum_buffer') is not None:
            out[name] = st['momentum_buffer'].detach().clone().float()
    return out
