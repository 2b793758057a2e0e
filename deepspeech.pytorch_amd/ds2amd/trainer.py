"""The training step of the reference (ref train.py:555-647 ``Trainer.train_batch``)
on the HIP path, with the reference's data-parallel semantics (train.py:804-809,
947-951; data/utils.py:40-44).

Per batch: input-size quirk (pct * T -> int, float32), forward, greedy decode,
NaN guard, CTC / N, zero_grad, backward with the bucketed gradient all-reduce
overlapped, clip_grad_norm_(max_norm) and SGD-Nesterov — the last two as one
device-resident pass with the NaN-skip decided on the device.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from . import _lib, ops
from .ctc import CTCLoss
from .decoder import GreedyDecoder
from .ops import _stream
from .optim import FlatParams, FusedSGD, GradAllReducer


def reduce_tensor(tensor, world_size):
    """data/utils.py:40-44: all-reduce SUM then divide by world size."""
    rt = tensor.clone()
    dist.all_reduce(rt, op=dist.ReduceOp.SUM)
    rt /= world_size
    return rt


def get_cer_wer(decoder, transcript, reference):
    """data/utils.py:47-57."""
    reference = reference.strip()
    transcript = transcript.strip()
    wer_ref = float(len(reference.split()) or 1)
    cer_ref = float(len(reference.replace(' ', '')) or 1)
    if reference == transcript:
        return 0, 0, wer_ref, cer_ref
    wer = decoder.wer(transcript, reference)
    cer = decoder.cer(transcript, reference)
    return wer, cer, wer_ref, cer_ref


class Trainer:
    """Owns the model's flat buffers, the fused optimizer and the gradient reducer."""

    def __init__(self, model, labels, lr=3e-4, momentum=0.9, max_norm=100.0, device=None,
                 bucket_mb=40.0, decode=True, score=False, group=None):
        self.device = torch.device(device) if device is not None else torch.device('cuda')
        self.model = model.to(self.device)
        self.model.train()
        self.flat = FlatParams(list(self.model.parameters()), self.device)
        self.optimizer = FusedSGD(self.flat, lr=lr, momentum=momentum, max_norm=max_norm)
        self.reducer = GradAllReducer(self.flat, bucket_mb=bucket_mb, group=group)
        self.world = self.reducer.world
        self.criterion = CTCLoss()
        self.decoder = GreedyDecoder(labels)
        self.decode = decode
        self.score = score
        self.nan_flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        # device accumulators of (wer, cer, words, chars): no host sync per batch
        self._score_acc = torch.zeros(4, dtype=torch.float64, device=self.device)

    # train.py:584-587 running sums, read lazily (one device->host copy)
    @property
    def train_wer(self):
        return float(self._score_acc[0])

    @property
    def train_cer(self):
        return float(self._score_acc[1])

    @property
    def num_words(self):
        return float(self._score_acc[2])

    @property
    def num_chars(self):
        return float(self._score_acc[3])

    def train_batch(self, data, return_item: bool = False):
        inputs, targets, filenames, input_percentages, target_sizes = data
        input_sizes = input_percentages.mul_(int(inputs.size(3))).int()   # train.py:557 quirk
        inputs = inputs.to(self.device, non_blocking=True)
        logits, probs, output_sizes = self.model(inputs, input_sizes)

        if self.decode:
            ids, offs, counts = self.decoder.decode_ids(probs, output_sizes)
            if self.score:
                self._score(ids, counts, targets, target_sizes)

        logits = logits.transpose(0, 1)                                   # T x N x C
        self.nan_flag.zero_()
        _lib.call("ds2_nan_guard", logits.data_ptr(), logits.numel(), 1,
                  self.nan_flag.data_ptr(), _stream())                    # train.py:595-598
        loss = self.criterion(logits, targets, output_sizes, target_sizes)
        loss = loss / inputs.size(0)

        self.optimizer.zero_grad()
        self.reducer.begin()
        loss.backward()
        self.reducer.finish()
        self.optimizer.step(skip_flag=self.nan_flag)                       # clip + SGD, NaN skip
        if self.world > 1:
            loss = reduce_tensor(loss.detach(), self.world)
        if return_item:
            v = float(loss.item())
            if v in (float('inf'), float('-inf')):
                v = 1000.0
            return v
        return loss.detach()

    def _score(self, ids, counts, targets, target_sizes):
        """get_cer_wer over the batch (train.py:575-587) on the device: ds2_edit_distance
        on the compact greedy ids vs the flat targets."""
        d, _ = ops.edit_distance_raw(ids, counts, targets, target_sizes, self.decoder.space_index)
        self._score_acc += d.sum(0, dtype=torch.float64)
