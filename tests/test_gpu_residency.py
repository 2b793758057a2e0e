"""GPU: residency of the persistent recurrences beside CUs held by a collective (cfg3's one
unverified assumption; reference DDP at train.py:947-951).

The recurrences are plain launches sized to one workgroup per CU whose workgroups spin on
each other's hand-offs: they finish only if every workgroup is resident at once.  At world > 1
an RCCL all-reduce overlapping the backward holds up to NCCL_MAX_NCHANNELS CUs, and
optim.GradAllReducer.guard_cooperative budgets for that.  Here a one-GPU stand-in holds CUs
the way the collective's CTAs would (ds2_test_occupy: one-wave workgroups with 96 KB of LDS,
alone on their CU, spinning on the device clock for a bounded time) and the device clock
(ds2_test_timestamp, s_memrealtime) orders what ran when:

* 32 CUs held (RCCL's cap), the cfg2 layer's 200-workgroup recurrences fit beside them: the
  guard does not wait, the recurrences run WHILE every occupier is resident, and the outputs
  and gradients are bit-identical to the run on an idle chip;
* 64 CUs held (200 + 64 > 256): the guard makes the compute stream wait for the occupier
  (registered like an in-flight bucket) before the backward recurrence starts -- outputs
  again bit-identical, no hand-off error;
* the launcher's LDS clamp (round 3's dispatch fault: 94 KB of static LDS + the 80 KB
  one-workgroup-per-CU pad exceeded the 160 KB per workgroup) keeps such a launch running.
"""
import time

import pytest
import torch

from ds2amd import _lib, ops
from ds2amd import model as dsm
from ds2amd.optim import FlatParams, GradAllReducer, _StreamDone

pytestmark = pytest.mark.gpu

T, N, H = 201, 32, 800          # cfg2's layer shape (T' shortened; the grid is T-independent)
HOLD_US = 1_500_000             # occupier bound: far longer than the layer's fwd + bwd


def _layer_and_inputs(dev):
    torch.manual_seed(4)
    layer = dsm.GRU(H, H, bidirectional=True).to(dev)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(T, N, H, generator=g).to(dev)
    dy = torch.randn(T, N, H, generator=g).to(dev)
    lens = torch.full((N,), T, dtype=torch.int32, device=dev)
    return layer, x, dy, lens


def _fwd(layer, x, lens):
    xr = x.clone().requires_grad_(True)
    y = layer.run(xr, lens, sum_dirs=True)
    return xr, y


def _bwd(layer, xr, y, dy):
    for p in layer.parameters():
        p.grad = None
    y.backward(dy)
    return [xr.grad.clone()] + [p.grad.clone() for p in layer.parameters()]


def _stamp(dev):
    t = torch.zeros(1, dtype=torch.int64, device=dev)
    _lib.call("ds2_test_timestamp", t.data_ptr(), ops._stream())
    return t


def _occupy(dev, ctas, stream):
    rec = torch.zeros(ctas * 4, dtype=torch.int64, device=dev)
    _lib.call("ds2_test_occupy", ctas, 96, HOLD_US, rec.data_ptr(), stream.cuda_stream)
    done = torch.cuda.Event()
    done.record(stream)
    return rec, done


def _reference(dev):
    layer, x, dy, lens = _layer_and_inputs(dev)
    xr, y = _fwd(layer, x, lens)
    grads = _bwd(layer, xr, y, dy)
    torch.cuda.synchronize()
    ops.check_rnn_status(dev)
    return layer, x, dy, lens, y.detach().clone(), grads


def test_recurrence_resident_beside_32_held_cus(dev):
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    grid = ops.persistent_bwd_grid("gru", N, H, 2)
    # the budget: the larger of the same-XCD x6 grid (200, what runs) and the direct-operand
    # fallback's 208 (the query never under-budgets)
    assert grid == 208, grid
    ctas = 32
    assert grid + ctas <= cus
    layer, x, dy, lens, y0, g0 = _reference(dev)
    flat = FlatParams(list(layer.parameters()), dev)
    red = GradAllReducer(flat, collective_ctas=ctas)
    side = torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    rec, done = _occupy(dev, ctas, side)
    time.sleep(0.05)                              # every occupier on its CU before we start
    red.begin()
    red.track(_StreamDone(done))
    ops.set_cooperative_guard(red.guard_cooperative)
    try:
        t0 = _stamp(dev)
        xr, y = _fwd(layer, x, lens)
        grads = _bwd(layer, xr, y, dy)
        t1 = _stamp(dev)
    finally:
        ops.set_cooperative_guard(None)
    torch.cuda.current_stream(dev).synchronize()  # the recurrences only; the occupier holds on
    assert red.guard_waits == 0
    torch.cuda.synchronize()
    ops.check_rnn_status(dev)
    r = rec.view(ctas, 4).cpu()
    starts, ends = r[:, 0], r[:, 1]
    # every occupier was resident before the layer began and still held its CU when it ended
    assert int(starts.max()) < int(t0.item()), (int(starts.max()), int(t0.item()))
    assert int(ends.min()) > int(t1.item()), (int(ends.min()), int(t1.item()))
    print(f"layer fwd+bwd {(int(t1.item()) - int(t0.item())) / 100:.0f} us beside {ctas} held CUs; "
          f"occupier XCC ids {sorted(set(r[:, 2].tolist()))}")
    assert torch.equal(y.detach(), y0)
    for a, b in zip(grads, g0):
        assert torch.equal(a, b)


def test_guard_waits_when_grid_plus_collective_exceeds_chip(dev):
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    grid = ops.persistent_bwd_grid("gru", N, H, 2)
    ctas = cus - grid + 8                         # 56 at cfg2: 208 + 56 > 256
    layer, x, dy, lens, y0, g0 = _reference(dev)
    flat = FlatParams(list(layer.parameters()), dev)
    red = GradAllReducer(flat, collective_ctas=ctas)
    xr, y = _fwd(layer, x, lens)                  # the forward on the idle chip (no collective
    torch.cuda.synchronize()                      # overlaps a forward in training)
    side = torch.cuda.Stream(dev)
    rec, done = _occupy(dev, ctas, side)
    time.sleep(0.05)
    red.begin()
    red.track(_StreamDone(done))
    after_guard = []

    def guard(g):
        red.guard_cooperative(g)
        after_guard.append(_stamp(dev))           # where the backward recurrence may start

    ops.set_cooperative_guard(guard)
    try:
        grads = _bwd(layer, xr, y, dy)
    finally:
        ops.set_cooperative_guard(None)
    torch.cuda.synchronize()
    ops.check_rnn_status(dev)
    assert red.guard_waits == 1
    assert len(after_guard) == 1
    ends = rec.view(ctas, 4)[:, 1].cpu()
    assert int(after_guard[0].item()) >= int(ends.max()), "the backward did not wait"
    assert torch.equal(y.detach(), y0)
    for a, b in zip(grads, g0):
        assert torch.equal(a, b)


def test_rnn_launch_clamps_lds_pad(dev):
    """A persistent-style launch with 94 KB of static LDS through the recurrences' launcher
    (rnn_launch, 80 KB pad): the pad is cut to what the static LDS leaves, the launch runs on
    every CU and finishes (round 3: the unclamped dispatch faulted)."""
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    rec = torch.zeros(cus * 4, dtype=torch.int64, device=dev)
    _lib.call("ds2_test_rnn_launch_lds", cus, 2000, rec.data_ptr(), ops._stream())
    torch.cuda.synchronize()
    r = rec.view(cus, 4).cpu()
    assert (r[:, 1] >= r[:, 0]).all() and (r[:, 0] > 0).all()   # every workgroup ran
    assert (r[:, 2] != -1).all()                                   # its static LDS held
