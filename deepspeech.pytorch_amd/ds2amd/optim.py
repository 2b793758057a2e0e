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

import ctypes
import os
from typing import List, Optional

import torch
import torch.distributed as dist

from . import _lib
from .ops import _stream, _p, register_grad_slot


class FlatParams:
    """Owns flat (param, grad, momentum) buffers; params/grads become views."""

    ALIGN = 64  # elements; keeps every view 256-byte aligned

    def __init__(self, params: List[torch.nn.Parameter], device, adjacent=(), tail: int = 0):
        """adjacent: (first, second) parameter pairs laid out back to back (first, then
        second, no padding between when first fills whole 64-element blocks) -- a
        bidirectional recurrent layer's W_ih of both directions, so its input projection,
        dX and dW_ih GEMMs run as one GEMM over both directions (ops._stacked_rows).
        tail: extra fp32 slots after the last parameter's gradient (``self.tail``), outside
        ``numel`` (no norm, clip or update touches them): the step's status word and loss ride
        in the last all-reduce bucket there (GradAllReducer, status_slots)."""
        params = [p for p in params if p.requires_grad]
        self.model_params = params                 # model.parameters() order
        order = list(reversed(params))             # backward-completion order
        second_of = {id(a): b for a, b in adjacent}
        seconds = {id(b) for _, b in adjacent}
        first_of = {id(b): a for a, b in adjacent}
        self.params = []
        placed = set()
        for p in order:
            if id(p) in placed:
                continue
            if id(p) in second_of or id(p) in seconds:
                a = p if id(p) in second_of else first_of[id(p)]
                b = second_of[id(a)]
                for q in (a, b):
                    self.params.append(q)
                    placed.add(id(q))
            else:
                self.params.append(p)
                placed.add(id(p))
        offs, total = [], 0
        for p in self.params:
            offs.append(total)
            total += (p.numel() + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.numel = total
        self.offsets = offs
        self.offset_of = {id(p): o for p, o in zip(self.params, offs)}
        self.tail_alloc = (tail + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.flat = torch.zeros(total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(total + self.tail_alloc, dtype=torch.float32, device=device)
        self.tail = self.grad[total:total + tail]
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
        self.steps = 0

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
        self.steps += 1

    # ---- torch.optim.SGD's state_dict format (model.py:446 optim_dict; train.py:843) ----
    def _model_order(self):
        """(param, flat offset) in the reference optimizer's order: model.parameters()
        (build_optimizer(args, model.parameters()), train.py:139-152, 939)."""
        return [(p, self.flat.offset_of[id(p)]) for p in self.flat.model_params]

    def _group_defaults(self):
        # the installed torch's own SGD param_group keys, so the dict loads into
        # torch.optim.SGD of this torch version unchanged
        probe = torch.optim.SGD([torch.zeros(1, requires_grad=True)], lr=self.lr,
                                momentum=self.momentum, nesterov=True)
        g = dict(probe.param_groups[0])
        g.pop('params')
        return g

    def state_dict(self):
        """torch.optim.SGD(model.parameters(), lr, momentum, nesterov=True).state_dict():
        per-parameter ``momentum_buffer`` (after the first step) in model.parameters()
        order and one param_group.  ``max_norm`` is train.py's --max-norm argument, not
        optimizer state, so it is not stored (as in the reference)."""
        order = self._model_order()
        state = {}
        if self.steps > 0:
            for i, (p, o) in enumerate(order):
                state[i] = {'momentum_buffer': self.buf[o:o + p.numel()].detach().view_as(p)
                            .cpu().clone()}
        group = self._group_defaults()
        group['params'] = list(range(len(order)))
        return {'state': state, 'param_groups': [group]}

    def load_state_dict(self, sd):
        """Accepts torch.optim.SGD's format (a reference ``package['optim_dict']``).  Raises
        on anything else instead of silently restarting the momentum."""
        if not isinstance(sd, dict) or set(sd) != {'state', 'param_groups'}:
            raise ValueError("FusedSGD.load_state_dict expects a torch.optim.SGD state_dict "
                             f"({{'state', 'param_groups'}}), got keys {sorted(sd) if isinstance(sd, dict) else type(sd)}")
        groups = sd['param_groups']
        order = self._model_order()
        if len(groups) != 1:
            raise ValueError(f"expected one param_group (model.parameters()), got {len(groups)}")
        g = groups[0]
        if len(g['params']) != len(order):
            raise ValueError(f"param_group holds {len(g['params'])} parameters, the model has "
                             f"{len(order)}")
        if not g.get('nesterov', False) or g.get('dampening', 0) != 0 or \
                g.get('weight_decay', 0) != 0 or g.get('maximize', False):
            raise ValueError("FusedSGD implements SGD(momentum, nesterov=True, dampening=0, "
                             "weight_decay=0) (train.py:146-149); the state_dict has "
                             f"nesterov={g.get('nesterov')}, dampening={g.get('dampening')}, "
                             f"weight_decay={g.get('weight_decay')}")
        self.lr = float(g['lr'])
        self.momentum = float(g['momentum'])
        self.buf.zero_()
        state = sd['state']
        for slot, idx in enumerate(g['params']):
            st = state.get(idx)
            if not st:
                continue
            unknown = set(st) - {'momentum_buffer'}
            if unknown:
                raise ValueError(f"unrecognised SGD state keys {sorted(unknown)} for param {idx}")
            mb = st.get('momentum_buffer')
            if mb is None:
                continue
            p, o = order[slot]
            if tuple(mb.shape) != tuple(p.shape):
                raise ValueError(f"momentum_buffer {idx}: shape {tuple(mb.shape)} != parameter "
                                 f"{tuple(p.shape)}")
            self.buf[o:o + p.numel()].copy_(mb.reshape(-1).to(self.buf.device, torch.float32))
        self.steps = max(self.steps, 1 if state else 0)


class ParamBroadcaster:
    """DistributedDataParallel's replica consistency (train.py:947-951): rank 0's parameters
    and buffers are broadcast once at construction, and (broadcast_buffers=True, DDP's
    default) rank 0's BatchNorm running statistics before every forward.

    The float buffers (running_mean / running_var, 32.5 KB at cfg2) are re-pointed into one
    flat tensor so the per-forward sync is ONE broadcast; num_batches_tracked (int64,
    identical on every rank: one increment per forward) is broadcast once at construction.
    """

    def __init__(self, model, flat: FlatParams, group=None, broadcast_buffers: bool = True):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.src = dist.get_global_rank(group, 0) if (group is not None and self.world > 1) else 0
        self.broadcast_buffers = broadcast_buffers
        bufs = [b for b in model.buffers() if b.is_floating_point()]
        self.others = [b for b in model.buffers() if not b.is_floating_point()]
        total = sum(b.numel() for b in bufs)
        dev = flat.flat.device
        self.flat_buffers = torch.zeros(total, dtype=torch.float32, device=dev)
        o = 0
        for b in bufs:
            n = b.numel()
            self.flat_buffers[o:o + n].copy_(b.data.reshape(-1))
            b.data = self.flat_buffers[o:o + n].view_as(b)
            o += n
        self.flat = flat
        self.broadcasts = 0
        if self.world > 1:
            dist.broadcast(flat.flat, self.src, group=group)
            dist.broadcast(self.flat_buffers, self.src, group=group)
            for b in self.others:
                dist.broadcast(b.data, self.src, group=group)
            self.broadcasts += 1

    def before_forward(self):
        if self.world > 1 and self.broadcast_buffers and self.flat_buffers.numel():
            dist.broadcast(self.flat_buffers, self.src, group=self.group)
            self.broadcasts += 1


UNKNOWN_CTAS = 1 << 30
_warned_uncapped = [False]


def rccl_channel_cap() -> int:
    """The CTA budget RCCL may hold while a persistent recurrence runs:
    NCCL_MAX_NCHANNELS, which init_distributed() sets to 32 before the communicator exists.
    Unset or unreadable (a process group created elsewhere: RCCL then picks its own channel
    count, which nothing here can read back) the budget is unknown: ``UNKNOWN_CTAS``, so the
    guard always waits for the buckets in flight before a persistent recurrence,
    and a warning says so once."""
    try:
        return int(os.environ["NCCL_MAX_NCHANNELS"])
    except (KeyError, ValueError):
        if not _warned_uncapped[0]:
            _warned_uncapped[0] = True
            import warnings
            warnings.warn("NCCL_MAX_NCHANNELS is not set: RCCL's CTA count is unknown, so every "
                          "persistent recurrence waits for the all-reduces in flight "
                          "(ds2amd.trainer.init_distributed caps it at 32)")
        return UNKNOWN_CTAS


def global_status_word(word: torch.Tensor, group=None) -> torch.Tensor:
    """Make a per-rank status word global, in place: MAX over the ranks (any rank's non-zero
    word becomes every rank's).  The step's skip decision must be one decision: a rank whose
    recurrence failed has already summed its NaN gradients into every rank's buckets, so
    every rank skips the update and every rank raises at the same step (no rank is left
    waiting in the next collective).  A no-op without a process group or at world 1."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(word, op=dist.ReduceOp.MAX, group=group)
    return word


class _StreamDone:
    """Completion of a collective enqueued on a side stream: ``wait()`` makes the current
    stream wait for it (no host sync), like an async torch.distributed work handle."""

    def __init__(self, event: torch.cuda.Event):
        self.event = event

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)


class RcclComm:
    """``ds2_comm_t``: this rank's RCCL communicator created through the C ABI
    (ds2_comm_get_unique_id on rank 0, the id carried to every rank by
    torch.distributed, ds2_comm_init), and ``all_reduce_async`` = ds2_allreduce_bucket
    on a dedicated communication stream ordered after the current stream's work so far
    (SURVEY §8b allreduce_bucket; replaces DDP's NCCL all-reduce, train.py:947-951)."""

    def __init__(self, group=None, device=None):
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        dev = torch.device("cuda") if device is None else torch.device(device)
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        nbytes = _lib.size("ds2_comm_id_bytes")
        uid = torch.zeros(nbytes, dtype=torch.uint8)
        if self.rank == 0:
            buf = ctypes.create_string_buffer(nbytes)
            _lib.call("ds2_comm_get_unique_id", ctypes.addressof(buf))
            uid = torch.frombuffer(bytearray(buf.raw), dtype=torch.uint8).clone()
        t = uid.to(dev) if dist.get_backend(group) == "nccl" else uid
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast(t, src, group=group)
        idbuf = ctypes.create_string_buffer(t.cpu().numpy().tobytes(), nbytes)
        self.handle = ctypes.c_void_p()
        _lib.call("ds2_comm_init", ctypes.addressof(self.handle), ctypes.addressof(idbuf),
                  self.world, self.rank, dev.index)
        self.stream = torch.cuda.Stream(dev)

    def all_reduce_async(self, bucket: torch.Tensor) -> _StreamDone:
        """In-place SUM of one contiguous fp32 bucket across the ranks."""
        ready = torch.cuda.Event()
        ready.record()
        self.stream.wait_event(ready)
        _lib.call("ds2_allreduce_bucket", self.handle.value, bucket.data_ptr(), bucket.numel(),
                  self.stream.cuda_stream)
        done = torch.cuda.Event()
        done.record(self.stream)
        return _StreamDone(done)

    def close(self):
        if self.handle.value:
            _lib.call("ds2_comm_destroy", self.handle.value)
            self.handle = ctypes.c_void_p()


class _Both:
    """Two in-flight handles waited as one (the all-reduce and its traffic stand-in)."""

    def __init__(self, a, b):
        self.a, self.b = a, b

    def wait(self):
        self.a.wait()
        self.b.wait()


class _Waited:
    """A handle the compute stream already waited for (the 'gap' policy): later waits on it
    cost nothing and are not counted again."""

    def __init__(self, h):
        self.h = h

    def wait(self):
        pass


class RingTrafficStandIn:
    """One-GPU stand-in for a ring all-reduce's local HBM traffic (DS2_AR_STANDIN=busbw_GBps
    [,world]): for a bucket of S bytes, ``ds2_test_ring_traffic`` runs the
    2 (W - 1) ring phases of an all-reduce over W ranks on a side stream, each phase reading
    an S / W chunk of the bucket and a chunk of scratch and writing the scratch chunk (the
    received data a peer lands in this GPU's HBM, reduced and passed on), paced so a phase
    lasts (S / W) / busbw, on ``ctas`` CUs (RCCL's channel cap).  The gradients are only read:
    results stay bit-identical.  Measurement only -- never on by default."""

    def __init__(self, spec: str, device, ctas: int = 32):
        parts = spec.split(",")
        self.busbw = float(parts[0])
        self.world = int(parts[1]) if len(parts) > 1 else 8
        self.ctas = ctas
        self.device = device
        self.stream = torch.cuda.Stream(device)
        self.scratch = None
        self.launches = 0

    def run(self, bucket: torch.Tensor):
        count = bucket.numel()
        # the kernel's chunk: ceil(floor(count / 4) / world) float4s (ds2_test_ring_traffic)
        chunk = 4 * ((count // 4 + self.world - 1) // self.world)
        if self.scratch is None or self.scratch.numel() < chunk:
            if self.scratch is not None:
                # the side stream may still be reading the old buffer
                torch.cuda.current_stream(self.device).wait_stream(self.stream)
            self.scratch = torch.zeros(chunk, dtype=torch.float32, device=self.device)
            self.scratch.record_stream(self.stream)
        ready = torch.cuda.Event()
        ready.record()
        self.stream.wait_event(ready)
        _lib.call("ds2_test_ring_traffic", bucket.data_ptr(), count, self.world,
                  self.scratch.data_ptr(), self.ctas, float(self.busbw), self.stream.cuda_stream)
        self.launches += 1
        done = torch.cuda.Event()
        done.record(self.stream)
        return _StreamDone(done)


class GradAllReducer:
    """Bucketed gradient all-reduce (SUM, then /world) overlapped with backward.

    Buckets are contiguous slices of the flat gradient buffer (fc/last RNN layers
    first).  A post-accumulate hook counts ready parameters per bucket; the
    moment a bucket is complete its all_reduce is issued asynchronously (RCCL
    over xGMI with backend 'nccl', gloo on CPU test rigs) while autograd keeps
    producing earlier layers' gradients.  ``finish()`` waits and applies 1/world
    (exact for power-of-two worlds, so it equals DDP's divide-then-sum bit for bit).

    CU budget: each recurrence's backward is ONE persistent launch (a plain launch sized to
    one workgroup per CU: 200 of 256 CUs at cfg2) whose workgroups spin on each other's
    hand-offs, so all of them must be resident at once; the hardware gives no such guarantee
    beside a collective that holds CUs.  ``guard_cooperative(grid)`` is called before each
    such launch; when the grid plus the CTAs the collectives in flight may hold
    (``collective_ctas``: RCCL's channel cap at world > 1) would not fit the chip, the compute
    stream first waits for the all-reduces already in flight (a stream wait, no host sync),
    so a collective never holds CUs a spinning recurrence needs.  ``collective_ctas`` can be
    given explicitly (the one-GPU residency test drives the guard at world 1 with an
    occupying kernel registered through ``track``).
    """

    def __init__(self, flat: FlatParams, bucket_mb: float = 40.0, group=None,
                 comm: Optional[RcclComm] = None, collective_ctas: Optional[int] = None,
                 policy: Optional[str] = None):
        """policy: when a bucket's all-reduce may run beside a persistent recurrence --
        'overlap' (default): issued the moment the bucket is complete, running beside
        whatever the backward does next; 'gap': each backward recurrence first waits for
        the all-reduces in flight (DS2_AR_POLICY; DESIGN.md §6 has the measured A/B).
        The last bucket also carries ``flat.tail`` (the status word and the loss, packed by
        the function given to ``set_status_packer``) when the flat buffer has one, so a step
        issues one series of collectives, not three."""
        self.flat = flat
        self.group = group
        self.comm = comm     # None: torch.distributed; else ds2_allreduce_bucket
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.policy = policy or os.environ.get("DS2_AR_POLICY", "overlap")
        if self.policy not in ("overlap", "gap"):
            raise ValueError(f"DS2_AR_POLICY must be 'overlap' or 'gap', got {self.policy!r}")
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
                if i + 1 == len(plist):
                    nxt = flat.numel + flat.tail_alloc     # the status tail rides along
                self._close(start, nxt, members)
                start, members = nxt, []
        self.pending = [0] * len(self.buckets)
        self.handles = [None] * len(self.buckets)
        self.issued_from_hooks = 0
        self.collectives = 0       # collectives issued in the last step
        self.guard_waits = 0
        self.cus = 0
        if flat.flat.is_cuda:
            self.cus = torch.cuda.get_device_properties(flat.flat.device).multi_processor_count
        if collective_ctas is None:
            collective_ctas = rccl_channel_cap() if self.world > 1 else 0
        self.rccl_ctas = int(collective_ctas)
        self.extra = []            # in-flight work registered by track()
        self._pack = None
        self._packed = False
        self.standin = None        # RingTrafficStandIn (DS2_AR_STANDIN), one-GPU measurements
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

    def set_status_packer(self, fn) -> None:
        """fn(tail) writes this step's status slots into ``flat.tail`` on the current stream;
        called right before the last bucket's all-reduce is issued (by then every recurrence
        of the backward has been enqueued: the last bucket holds the conv block's
        parameters, whose gradients come last)."""
        self._pack = fn

    def begin(self):
        self.pending = [b[2] for b in self.buckets]
        self.handles = [None] * len(self.buckets)
        self.issued_from_hooks = 0
        self.collectives = 0
        self._packed = False
        self.extra = []

    def track(self, handle):
        """Register other in-flight work that may hold CUs (an object with ``wait()`` that
        makes the current stream wait for it): the guard waits for it like a bucket."""
        self.extra.append(handle)

    def _on_ready(self, p):
        self.flat.adopt(p, self.param_offset[id(p)])
        b = self.param_bucket[id(p)]
        self.pending[b] -= 1
        if self.pending[b] == 0:
            self.handles[b] = self._issue(b)
            self.issued_from_hooks += 1

    def _issue(self, b):
        s, e, _ = self.buckets[b]
        if b == len(self.buckets) - 1 and self._pack is not None and not self._packed:
            self._pack(self.flat.tail)
            self._packed = True
        self.collectives += 1
        bucket = self.flat.grad[s:e]
        h = self._all_reduce(bucket)
        if self.standin is not None:
            h = _Both(h, self.standin.run(bucket))
        return h

    def _all_reduce(self, bucket):
        if self.comm is not None:
            return self.comm.all_reduce_async(bucket)
        return dist.all_reduce(bucket, group=self.group, async_op=True)

    def guard_cooperative(self, grid: int):
        if self.policy != "gap":
            if self.cus <= 0 or self.rccl_ctas <= 0:
                return
            if min(grid, self.cus) + self.rccl_ctas <= self.cus:
                return
        for i, h in enumerate(list(self.handles) + self.extra):
            if h is not None and not isinstance(h, _Waited):
                h.wait()
                self.guard_waits += 1
                if i < len(self.handles):
                    self.handles[i] = _Waited(h)

    def finish(self):
        if not self._hooks:
            return
        self.flat.finalize_grads()   # zero the slices no gradient was written to
        for b, h in enumerate(self.handles):
            if h is None:     # a bucket whose params received no gradient this step
                h = self._issue(b)
            h.wait()
        if self.world > 1:
            self.flat.grad.mul_(1.0 / self.world)
