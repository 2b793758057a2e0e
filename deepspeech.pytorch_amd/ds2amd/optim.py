"""Training-step tail: flat parameter/gradient buffers, fused clip + SGD-Nesterov,
and the data-parallel gradient exchange.

ref train.py:139-152 (SGD, momentum 0.9, nesterov=True, weight_decay 0),
train.py:619-632 (zero_grad, backward, clip_grad_norm_(max_norm), NaN-skip, step),
train.py:947-951 (DistributedDataParallel) and data/utils.py:40-44 (reduce_tensor).

Parameters are re-pointed into one flat fp32 buffer laid out in *reverse*
registration order (fc first, conv last) — the order autograd finishes their
gradients — and every ``p.grad`` is a view of a matching flat gradient buffer,
so (a) the gradient norm, clip and Nesterov update are two kernel launches over
the whole model (ds2_grad_norm, ds2_clip_sgd_nesterov; norm never leaves the
device) and (b) the all-reduce buckets are contiguous slices that become ready
front to back while backward is still running.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from . import _lib
from .ops import _stream, _p, register_grad_slot


class FlatParams:
    """Owns flat (param, grad, momentum) buffers; params/grads become views."""

    ALIGN = 64  # elements; keeps every view 256-byte aligned

    def __init__(self, params: List[torch.nn.Parameter], device):
        params = [p for p in params if p.requires_grad]
        self.params = list(reversed(params))       # backward-completion order
        offs, total = [], 0
        for p in self.params:
            offs.append(total)
            total += (p.numel() + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.numel = total
        self.offsets = offs
        self.flat = torch.zeros(total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(total, dtype=torch.float32, device=device)
        for p, o in zip(self.params, offs):
            n = p.numel()
            self.flat[o:o + n].copy_(p.data.reshape(-1))
            p.data = self.flat[o:o + n].view_as(p)
            p.grad = self.grad[o:o + n].view_as(p)
            register_grad_slot(p, self.grad, o)

    def zero_grad(self):
        """set_to_none semantics (torch's default): the next backward writes every
        parameter gradient straight into its slice (ops.grad_like) and autograd adopts
        the view, so no memset and no accumulate kernels.  finalize_grads() zeroes the
        slices of parameters that received no gradient."""
        for p in self.params:
            p.grad = None

    def adopt(self, p, o):
        """Make p.grad the view of its slice: zero it when no gradient arrived, copy a
        gradient that some other op (not ops.grad_like) produced elsewhere."""
        n = p.numel()
        slot = self.grad[o:o + n]
        g = p.grad
        if g is None:
            slot.zero_()
        elif g.data_ptr() != slot.data_ptr():
            slot.copy_(g.reshape(-1))
        else:
            return
        p.grad = slot.view_as(p)

    def finalize_grads(self):
        for p, o in zip(self.params, self.offsets):
            self.adopt(p, o)

    def slices(self):
        for p, o in zip(self.params, self.offsets):
            yield p, o, p.numel()


class FusedSGD:
    """torch.optim.SGD(lr, momentum, nesterov=True) + clip_grad_norm_ on flat buffers."""

    def __init__(self, flat: FlatParams, lr: float, momentum: float = 0.9,
                 max_norm: float = 0.0, nesterov: bool = True):
        if not nesterov:
            raise ValueError("FusedSGD implements the reference's nesterov=True update")
        self.flat = flat
        self.lr = lr
        self.momentum = momentum
        self.max_norm = max_norm
        dev = flat.flat.device
        self.buf = torch.zeros_like(flat.flat)
        self.norm = torch.zeros(1, dtype=torch.float32, device=dev)
        self.skip = torch.zeros(1, dtype=torch.int32, device=dev)
        self.ws = torch.empty(max(16, _lib.size("ds2_optim_workspace_size", flat.numel)),
                              dtype=torch.uint8, device=dev)

    def zero_grad(self):
        self.flat.zero_grad()

    def grad_norm(self) -> torch.Tensor:
        """Global L2 norm of the gradients, on the device (no host sync)."""
        self.flat.finalize_grads()
        _lib.call("ds2_grad_norm", self.flat.grad.data_ptr(), self.flat.numel, self.norm.data_ptr(),
                  self.ws.data_ptr(), self.ws.numel(), _stream())
        return self.norm

    def step(self, skip_flag: Optional[torch.Tensor] = None):
        self.flat.finalize_grads()
        norm_ptr = None
        if self.max_norm > 0:
            self.grad_norm()
            norm_ptr = self.norm.data_ptr()
        _lib.call("ds2_clip_sgd_nesterov", self.flat.flat.data_ptr(), self.flat.grad.data_ptr(),
                  self.buf.data_ptr(), self.flat.numel, float(self.lr), float(self.momentum),
                  float(self.max_norm), norm_ptr, _p(skip_flag), _stream())

    def state_dict(self):
        return {"lr": self.lr, "momentum": self.momentum, "max_norm": self.max_norm,
                "momentum_buffer": self.buf.detach().cpu()}

    def load_state_dict(self, sd):
        self.lr = sd.get("lr", self.lr)
        self.momentum = sd.get("momentum", self.momentum)
        self.max_norm = sd.get("max_norm", self.max_norm)
        if "momentum_buffer" in sd:
            self.buf.copy_(sd["momentum_buffer"].to(self.buf.device))


class GradAllReducer:
    """Bucketed gradient all-reduce (SUM, then /world) overlapped with backward.

    Buckets are contiguous slices of the flat gradient buffer (fc/last RNN layers
    first).  A post-accumulate hook counts ready parameters per bucket; the
    moment a bucket is complete its all_reduce is issued asynchronously (RCCL
    over xGMI with backend 'nccl', gloo on CPU test rigs) while autograd keeps
    producing earlier layers' gradients.  ``finish()`` waits and applies 1/world.
    """

    def __init__(self, flat: FlatParams, bucket_mb: float = 40.0, group=None):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        cap = int(bucket_mb * 1024 * 1024 / 4)
        self.buckets = []          # (start, end, n_params) element ranges
        self.param_bucket = {}
        start, members = 0, []
        plist = list(flat.slices())
        self.param_offset = {id(p): o for p, o, _ in plist}
        for i, (p, o, n) in enumerate(plist):
            members.append(p)
            nxt = plist[i + 1][1] if i + 1 < len(plist) else flat.numel
            if nxt - start >= cap or i + 1 == len(plist):
                self._close(start, nxt, members)
                start, members = nxt, []
        self.pending = [0] * len(self.buckets)
        self.handles = [None] * len(self.buckets)
        self._hooks = []
        # hooks whenever a process group exists (world 1 included: that exercises the
        # RCCL path on a single-GPU box; the all-reduce is then a no-op copy)
        if dist.is_initialized():
            for p in flat.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_ready))

    def _close(self, start, end, members):
        b = len(self.buckets)
        self.buckets.append((start, end, len(members)))
        for p in members:
            self.param_bucket[id(p)] = b

    def begin(self):
        self.pending = [b[2] for b in self.buckets]
        self.handles = [None] * len(self.buckets)

    def _on_ready(self, p):
        self.flat.adopt(p, self.param_offset[id(p)])
        b = self.param_bucket[id(p)]
        self.pending[b] -= 1
        if self.pending[b] == 0:
            s, e, _ = self.buckets[b]
            self.handles[b] = dist.all_reduce(self.flat.grad[s:e], group=self.group,
                                              async_op=True)

    def finish(self):
        if not self._hooks:
            return
        self.flat.finalize_grads()   # zero the slices no gradient was written to
        for b, h in enumerate(self.handles):
            if h is None:     # a bucket whose params received no gradient this step
                s, e, _ = self.buckets[b]
                h = dist.all_reduce(self.flat.grad[s:e], group=self.group, async_op=True)
            h.wait()
        if self.world > 1:
            self.flat.grad.mul_(1.0 / self.world)
