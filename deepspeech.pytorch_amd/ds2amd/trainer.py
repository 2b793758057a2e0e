"""The training step of the reference (ref train.py:555-647 ``Trainer.train_batch``)
on the HIP path, with the reference's data-parallel semantics (train.py:804-809,
947-951; data/utils.py:40-44).

Per batch: input-size quirk (pct * T -> int, float32), forward, greedy decode (+ the
per-batch CER/WER of train.py:575-587 on the device), the NaN work-around of
train.py:595-598 (NaN logits zeroed in place, their gradient zero, the step always
taken -- the reference's skip check at :625 can never fire after :598), CTC / N,
zero_grad, backward with the bucketed gradient all-reduce overlapped,
clip_grad_norm_(max_norm) and SGD-Nesterov as one device-resident pass.

No host synchronisation per step: the reference's two warnings (NaN logits, inf loss)
and the persistent recurrences' hand-off status (ds2hip.h err_out) travel to the host
in a small pinned ring and are read once the GPU has finished that step -- at the next
``train_batch``, in ``poll_status(block=True)``, or when ``return_item=True`` asks for
the loss value anyway.  A hand-off failure raises ``Ds2Error``.
"""
from __future__ import annotations

import os
from collections import deque
from typing import Optional

import torch
import torch.distributed as dist

from . import _lib, ops
from .ctc import CTCLoss
from .decoder import GreedyDecoder
from .ops import _stream
from .optim import FlatParams, FusedSGD, GradAllReducer, ParamBroadcaster, RcclComm


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


def init_distributed(backend: str = "nccl", device_id: Optional[int] = None):
    """One process per GPU (torch.distributed.run env).  Before the communicator exists,
    cap RCCL's channels (= CTAs it may hold) at 32 unless the user chose otherwise, so an
    all-reduce overlapping the backward always leaves the persistent recurrence its 208
    co-resident workgroups."""
    os.environ.setdefault("NCCL_MAX_NCHANNELS", "32")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    local = int(os.environ.get("LOCAL_RANK", "0")) if device_id is None else device_id
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return local


class _ZeroNaN(torch.autograd.Function):
    """train.py:595-598 ``logits[torch.isnan(logits)] = 0`` as an in-place op: NaNs become 0
    (ds2_nan_guard, which also sets the step's flag and records a byte mask) and, as for
    autograd's index_put, the zeroed positions pass no gradient (ds2_zero_masked, a no-op
    unless the flag is set)."""

    @staticmethod
    def forward(ctx, x, flag, mask):
        _lib.call("ds2_nan_guard", x.data_ptr(), x.numel(), 1, flag.data_ptr(), mask.data_ptr(),
                  _stream())
        ctx.mark_dirty(x)
        ctx.save_for_backward(flag, mask)
        return x

    @staticmethod
    def backward(ctx, g):
        flag, mask = ctx.saved_tensors
        g = g.contiguous().clone()
        _lib.call("ds2_zero_masked", g.data_ptr(), mask.data_ptr(), g.numel(), flag.data_ptr(),
                  _stream())
        return g, None, None


class Trainer:
    """Owns the model's flat buffers, the fused optimizer and the gradient reducer."""

    STATUS_RING = 4

    def __init__(self, model, labels, lr=3e-4, momentum=0.9, max_norm=100.0, device=None,
                 bucket_mb=40.0, decode=True, score=False, group=None, broadcast_buffers=True,
                 verbose=True):
        self.device = torch.device(device) if device is not None else torch.device('cuda')
        self.model = model.to(self.device)
        self.model.train()
        # both directions' W_ih of a bidirectional recurrent layer back to back: one GEMM
        # per layer for the input projection, dX and dW_ih (ops._stacked_rows)
        pairs = [(m.weight_ih_l0, m.weight_ih_l0_reverse) for m in self.model.modules()
                 if hasattr(m, 'weight_ih_l0_reverse')]
        # two tail slots after the gradients: (status word, loss), all-reduced with the last
        # bucket (GradAllReducer.set_status_packer) instead of two collectives of their own
        self.flat = FlatParams(list(self.model.parameters()), self.device, adjacent=pairs,
                               tail=2 if dist.is_initialized() else 0)
        self.optimizer = FusedSGD(self.flat, lr=lr, momentum=momentum, max_norm=max_norm)
        # DS2_ALLREDUCE=ds2: the buckets go through the library's own RCCL communicator
        # (ds2_comm_init / ds2_allreduce_bucket) instead of torch.distributed's
        comm = None
        if (dist.is_initialized() and self.device.type == "cuda"
                and os.environ.get("DS2_ALLREDUCE", "torch") == "ds2"):
            comm = RcclComm(group, self.device)
        self.reducer = GradAllReducer(self.flat, bucket_mb=bucket_mb, group=group, comm=comm)
        self.world = self.reducer.world
        if dist.is_initialized():
            self.reducer.set_status_packer(self._pack_status)
            spec = os.environ.get("DS2_AR_STANDIN")
            if spec and self.device.type == "cuda":
                from .optim import RingTrafficStandIn
                self.reducer.standin = RingTrafficStandIn(spec, self.device,
                                                          ctas=self.reducer.rccl_ctas or 32)
        self._step_loss = None
        # DDP: rank 0's parameters and buffers everywhere (construction), rank 0's BN running
        # statistics before every forward (broadcast_buffers, train.py:950-951)
        self.sync = ParamBroadcaster(self.model, self.flat, group=group,
                                     broadcast_buffers=broadcast_buffers)
        if dist.is_initialized():
            ops.set_cooperative_guard(self.reducer.guard_cooperative)
        self.criterion = CTCLoss()
        self.decoder = GreedyDecoder(labels)
        self.decode = decode
        self.score = score
        self.verbose = verbose
        self.nan_flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._nan_mask = None
        # device accumulators of (wer, cer, words, chars): no host sync per batch
        self._score_acc = torch.zeros(4, dtype=torch.float64, device=self.device)
        # greedy decode + CER/WER depend on the forward alone: they run on a side stream
        # beside the CTC / backward (the recurrences leave CUs idle) and are joined before
        # the step ends
        self._side = torch.cuda.Stream(device=self.device) if self.device.type == 'cuda' else None
        self._rnn_word = ops.rnn_status_word(self.device)
        # pinned ring of (nan flag, rnn status, loss bits, global status bits) per in-flight step
        self._ring = [torch.zeros(4, dtype=torch.int32).pin_memory()
                      for _ in range(self.STATUS_RING)]
        self._ring_next = 0
        self._inflight = deque()
        self._status = torch.zeros(4, dtype=torch.int32, device=self.device)
        self.warnings = {"nan": 0, "inf_loss": 0}

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

    # ---- deferred status --------------------------------------------------------------
    def _pack_status(self, tail):
        """The last bucket's tail slots (GradAllReducer.set_status_packer): whether this
        rank's recurrence status word is non-zero (a FLAG, 1.0 or 0.0, not the bitmask: summed
        over the ranks it is non-zero iff any rank failed, whatever bits a word carries; each
        rank decodes its own word from ``_rnn_word``) and its loss (summed, then scaled by
        1/world with the gradients: reduce_tensor, data/utils.py:40-44)."""
        tail[0:1].copy_(self._rnn_word != 0)
        tail[1:2].copy_(self._step_loss)

    def _record_status(self, loss, global_word=None):
        """Stage (nan flag, recurrence status, loss bits, global status bits) of this step
        for the host."""
        st = self._status
        st[0:1].copy_(self.nan_flag)
        st[1:2].copy_(self._rnn_word)
        st[2:3].copy_(loss.detach().reshape(1).view(torch.int32))
        if global_word is not None:
            st[3:4].copy_(global_word)
        if len(self._inflight) == self.STATUS_RING:
            self._drain_one(block=True)
        buf = self._ring[self._ring_next]
        self._ring_next = (self._ring_next + 1) % self.STATUS_RING
        buf.copy_(st, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._inflight.append((ev, buf))

    def _drain_one(self, block: bool) -> bool:
        ev, buf = self._inflight[0]
        if not block and not ev.query():
            return False
        ev.synchronize()
        self._inflight.popleft()
        nan, err, loss_bits, global_bits = (int(v) for v in buf.tolist())
        loss = torch.tensor([loss_bits], dtype=torch.int32).view(torch.float32).item()
        msg = ops.rnn_status_error(err)
        if msg is None and global_bits != 0:
            msg = ("recurrence kernel failure on another rank (its NaN gradients were "
                   "all-reduced; every rank skipped the update)")
        if msg is not None:
            self._rnn_word.zero_()
            raise _lib.Ds2Error(msg)
        if nan:
            self.warnings["nan"] += 1
            if self.verbose:
                print("WARNING: Working around NaNs in data")          # train.py:597
        if loss in (float('inf'), float('-inf')):
            self.warnings["inf_loss"] += 1
            if self.verbose:
                print("WARNING: received an inf loss, setting loss value to 1000")   # :608
        return True

    def poll_status(self, block: bool = False) -> None:
        """Read the status of finished steps (all in-flight steps with block=True); raises
        Ds2Error if a recurrence kernel reported a hand-off failure."""
        while self._inflight and self._drain_one(block):
            pass

    def close(self) -> None:
        """Finish pending work and release the library's own RCCL communicator (DS2_ALLREDUCE=ds2;
        a no-op otherwise).  Call before destroying the process group."""
        if self.reducer.comm is not None:
            torch.cuda.synchronize(self.device)
            self.reducer.comm.close()
            self.reducer.comm = None

    # ---- the step ---------------------------------------------------------------------
    def train_batch(self, data, return_item: bool = False):
        self.poll_status(block=False)
        inputs, targets, filenames, input_percentages, target_sizes = data
        input_sizes = input_percentages.mul_(int(inputs.size(3))).int()   # train.py:557 quirk
        inputs = inputs.to(self.device, non_blocking=True)
        side = self._side if self.decode else None
        if side is not None and self.score:
            with torch.cuda.stream(side):      # idle stream: the host copies do not wait
                tg_d = targets.to(self.device, torch.int32, non_blocking=True)
                ts_d = target_sizes.to(self.device, torch.int32, non_blocking=True)
        self.sync.before_forward()
        logits, probs, output_sizes = self.model(inputs, input_sizes)

        if side is not None:
            main = torch.cuda.current_stream(self.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                ids, offs, counts = self.decoder.decode_ids(probs, output_sizes)
                if self.score:
                    self._score(ids, counts, tg_d, ts_d)
            for t in (probs, output_sizes):
                if torch.is_tensor(t) and t.is_cuda:
                    t.record_stream(side)

        logits = logits.transpose(0, 1)                                   # T x N x C
        self.nan_flag.zero_()
        if self._nan_mask is None or self._nan_mask.numel() < logits.numel():
            self._nan_mask = torch.empty(logits.numel(), dtype=torch.uint8, device=self.device)
        logits = _ZeroNaN.apply(logits, self.nan_flag, self._nan_mask)    # train.py:595-598
        loss = self.criterion(logits, targets, output_sizes, target_sizes)
        loss = loss / inputs.size(0)

        self.optimizer.zero_grad()
        self.reducer.begin()
        self._step_loss = loss.detach().reshape(1)
        loss.backward()
        self.reducer.finish()
        # clip + SGD; always taken for NaN data (see module docstring).  Skipped on the device
        # when a persistent recurrence reported a hand-off failure this step: its outputs are
        # NaN and the update would write NaN into every parameter and momentum slot before the
        # host sees the error (the word is 0 in a normal step; no host sync).  With a process
        # group the decision is global: the status word rode in the last gradient bucket's
        # tail, summed over the ranks (the failing rank's NaN gradients are already in every
        # rank's buckets, so all ranks skip and all raise), and so did the loss (reduce_tensor,
        # data/utils.py:40-44): one series of collectives per step.  A non-zero float sum has
        # non-zero bits, so the kernel reads the slot as its int skip flag.
        global_word = None
        if self.flat.tail.numel():
            global_word = self.flat.tail[0:1].view(torch.int32)
            self.optimizer.step(skip_flag=global_word)
            loss = self.flat.tail[1:2].clone().reshape(())
        else:
            self.optimizer.step(skip_flag=self._rnn_word)
        if side is not None:
            torch.cuda.current_stream(self.device).wait_stream(side)
        self._record_status(loss, global_word)
        if return_item:
            self.poll_status(block=True)
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
