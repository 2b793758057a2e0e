"""CPU (gloo, world_size 2): the data-parallel gradient exchange and sharding logic.

The HIP training step runs the same GradAllReducer over RCCL ('nccl') on the GPU
box; here the bucketing/hook/averaging logic is exercised with gloo on CPU
tensors: the averaged per-rank gradients must equal the single-process gradient
of the mean loss over the concatenated batch (DDP semantics, train.py:947-951).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ds2amd.optim import FlatParams, GradAllReducer
from ds2amd.data_loader import DistributedBucketingSampler


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(7, 33), torch.nn.Tanh(), torch.nn.Linear(33, 5),
                               torch.nn.Tanh(), torch.nn.Linear(5, 3))


def _data():
    g = torch.Generator().manual_seed(1)
    return torch.randn(8, 7, generator=g), torch.randn(8, 3, generator=g)


def _worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = _model()
    flat = FlatParams(list(m.parameters()), "cpu")
    red = GradAllReducer(flat, bucket_mb=0.0005)       # tiny buckets -> several buckets
    assert len(red.buckets) > 1
    x, y = _data()
    xs, ys = x[rank::world], y[rank::world]
    for step in range(2):
        flat.zero_grad()
        red.begin()
        loss = ((m(xs) - ys) ** 2).sum(1).mean()
        loss.backward()
        issued = sum(h is not None for h in red.handles)
        red.finish()
        if step == 1:
            # numpy copies travel by value (torch tensors would go through shm handles
            # that die with this process)
            out_q.put((rank, issued, len(red.buckets), flat.grad.numpy().copy(),
                       [p.grad.numpy().copy() for p in m.parameters()]))
    dist.destroy_process_group()


def test_grad_allreduce_matches_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m = _model()
    x, y = _data()
    # mean over ranks of per-rank mean losses == mean over the interleaved shards
    loss = sum(((m(x[r::world]) - y[r::world]) ** 2).sum(1).mean() for r in range(world)) / world
    loss.backward()
    ref = [p.grad for p in m.parameters()]
    for rank, issued, nb, flatg, grads in res:
        assert issued == nb, "every bucket's all-reduce was launched from the backward hooks"
        for g, r in zip(grads, ref):
            torch.testing.assert_close(torch.from_numpy(g), r, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(torch.from_numpy(res[0][3]), torch.from_numpy(res[1][3]))


def test_distributed_bucketing_sampler_matches_reference_semantics():
    data = list(range(23))
    bs, world = 4, 3
    bins = [list(range(i, min(i + bs, 23))) for i in range(0, 23, bs)]     # 6 bins
    total = 2 * world                                                       # ceil(6/3)*3
    padded = bins + bins[:total - len(bins)]
    for r in range(world):
        s = DistributedBucketingSampler(data, batch_size=bs, num_replicas=world, rank=r)
        assert list(s) == padded[r::world]
        assert len(s) == 2
    # uneven: 6 bins over 4 replicas -> padded to 8 by repeating the first bins
    s = DistributedBucketingSampler(data, batch_size=bs, num_replicas=4, rank=3)
    assert list(s) == (bins + bins[:2])[3::4]
    s0 = DistributedBucketingSampler(data, batch_size=bs, num_replicas=world, rank=0)
    s1 = DistributedBucketingSampler(data, batch_size=bs, num_replicas=world, rank=0)
    s0.shuffle(5)
    s1.shuffle(5)
    assert list(s0) == list(s1)              # epoch-seeded, identical on every rank


class _BNNet(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(4, 6)
        self.bn = torch.nn.BatchNorm1d(6)

    def forward(self, x):
        return self.bn(self.lin(x))


def _bcast_worker(rank, world, port, out_q):
    from ds2amd.optim import ParamBroadcaster
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(100 + rank)                 # deliberately different replicas
    m = _BNNet()
    m.bn.running_mean.fill_(float(rank + 1))
    flat = FlatParams(list(m.parameters()), "cpu")
    sync = ParamBroadcaster(m, flat)
    after_init = [p.detach().numpy().copy() for p in m.parameters()]
    rm0 = m.bn.running_mean.numpy().copy()
    m.train()
    g = torch.Generator().manual_seed(rank)       # different data per rank
    m(torch.randn(8, 4, generator=g))             # local BN stats diverge here
    sync.before_forward()                         # DDP: rank 0's buffers win before a forward
    out_q.put((rank, after_init, rm0, m.bn.running_mean.numpy().copy(),
               m.bn.running_var.numpy().copy(), int(m.bn.num_batches_tracked)))
    dist.destroy_process_group()


def test_param_broadcaster_matches_ddp_semantics():
    """DistributedDataParallel (train.py:947-951): rank 0's parameters and buffers are
    broadcast at construction; rank 0's BN running stats before every forward
    (broadcast_buffers=True)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, p0, rm0_0, rm_0, rv_0, nb0), (_, p1, rm0_1, rm_1, rv_1, nb1) = res
    for a, b in zip(p0, p1):
        assert (a == b).all()
    assert (rm0_0 == 1.0).all() and (rm0_1 == 1.0).all()     # rank 0's buffer everywhere
    assert (rm_0 == rm_1).all() and (rv_0 == rv_1).all()
    assert nb0 == nb1 == 1


# ---------------------------------------------------------------- the real DS2 layout
LABELS = "_'ABCDEFGHIJKLMNOPQRSTUVWXYZ2 "
CONF = dict(sample_rate=16000, window_size=0.02, window_stride=0.01, window='hamming')


def _ds2_params():
    from ds2amd import model as dsm
    torch.manual_seed(123456)
    m = dsm.DeepSpeech(rnn_type='gru', labels=LABELS, rnn_hidden_size=800, nb_layers=5,
                       audio_conf=CONF, bidirectional=True)
    return m


def _ds2_pairs(m):
    """The Trainer's adjacent pairs: both directions' W_ih of every bidirectional layer."""
    return [(mm.weight_ih_l0, mm.weight_ih_l0_reverse) for mm in m.modules()
            if hasattr(mm, 'weight_ih_l0_reverse')]


def _rank_grads(params, rank):
    g = torch.Generator().manual_seed(1000 + rank)
    return [torch.randn(p.shape, generator=g) for p in params]


def _ds2_worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = _ds2_params()
    params = [p for p in m.parameters() if p.requires_grad]
    flat = FlatParams(params, "cpu", adjacent=_ds2_pairs(m))
    red = GradAllReducer(flat, bucket_mb=40.0)
    grads = _rank_grads(params, rank)
    flat.zero_grad()
    red.begin()
    # injected per-rank gradients through autograd, so every parameter's post-accumulate
    # hook fires as in the real backward (the HIP ops write into the flat slots instead)
    loss = sum((p * g).sum() for p, g in zip(params, grads))
    loss.backward()
    issued = red.issued_from_hooks
    in_flight = sum(h is not None for h in red.handles)
    # CU budget: the 200-workgroup persistent backward plus the
    # 32-CTA cap init_distributed sets fits 256 CUs -> no wait; with no cap set the budget
    # is RCCL's 64 (rccl_channel_cap) and 200 + 64 does not fit -> the compute stream waits
    # for every all-reduce in flight
    from ds2amd.optim import rccl_channel_cap
    assert red.rccl_ctas == rccl_channel_cap()
    red.cus = 256
    red.rccl_ctas = 32
    red.guard_cooperative(200)
    waits_fit = red.guard_waits
    red.rccl_ctas = 64
    red.guard_cooperative(200)
    waits_over = red.guard_waits
    red.finish()
    out_q.put((rank, red.buckets, flat.offsets, [p.numel() for p in flat.params], flat.numel,
               issued, in_flight, waits_fit, waits_over, flat.grad.numpy().copy()))
    dist.destroy_process_group()


def test_grad_allreduce_real_ds2_layout():
    """GradAllReducer over the real DeepSpeech(5 x BiGRU-800) parameter list (41.2 M
    parameters, 164.8 MB flat, reverse layer order) with the bench's 40 MB buckets, gloo
    world 2: bucket boundaries fall on the first parameter boundary at or past 40 MB, every
    bucket is issued from the backward hooks, the result is the 1/W average of the ranks'
    gradients (train.py:947-951, data/utils.py:40-44), and the CU-budget guard waits only
    when the cooperative grid plus RCCL's CTA cap exceeds the chip."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ds2_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m = _ds2_params()
    params = [p for p in m.parameters() if p.requires_grad]
    assert sum(p.numel() for p in params) > 41_000_000
    layout = FlatParams(params, "cpu", adjacent=_ds2_pairs(m))
    cap = 40 * 1024 * 1024 // 4
    expect = None
    for rank, buckets, offs, sizes, numel, issued, in_flight, waits_fit, waits_over, g in res:
        # boundaries: contiguous, cover the flat buffer, close at the first parameter
        # boundary at or past the cap
        assert buckets[0][0] == 0 and buckets[-1][1] == numel
        bounds = offs[1:] + [numel]
        for i, (s_, e, n) in enumerate(buckets):
            assert e in bounds and n >= 1
            if i + 1 < len(buckets):
                assert buckets[i + 1][0] == e
                assert e - s_ >= cap
                prev = [b for b in bounds if s_ < b < e]
                assert all(b - s_ < cap for b in prev)
        assert len(buckets) == 4, [(b[1] - b[0]) * 4 / 2**20 for b in buckets]
        assert sum(b[2] for b in buckets) == len(sizes)
        assert issued == len(buckets) and in_flight == len(buckets)
        assert waits_fit == 0 and waits_over == len(buckets)
        if expect is None:
            # (g0 + g1) / 2 in the flat layout (reverse registration order, W_ih pairs
            # back to back)
            assert offs == layout.offsets
            g0 = _rank_grads(params, 0)
            g1 = _rank_grads(params, 1)
            expect = torch.zeros(numel)
            for p_, a, b in zip(params, g0, g1):
                o = layout.offset_of[id(p_)]
                expect[o:o + p_.numel()] = ((a + b) * 0.5).reshape(-1)
        assert torch.equal(torch.from_numpy(g), expect)


def test_flat_params_stacks_w_ih_pairs():
    """FlatParams with the Trainer's pairs: each bidirectional layer's W_ih (and its gradient
    slot) lies back to back, so ops._stacked_rows sees [W_ih_f; W_ih_r] as one matrix; every
    other parameter keeps the reverse registration order, and the optimizer's state order is
    still model.parameters() (torch.optim.SGD's)."""
    from ds2amd import ops
    from ds2amd.optim import FusedSGD
    torch.manual_seed(3)
    from ds2amd import model as dsm
    m = dsm.DeepSpeech(rnn_type="gru", labels=LABELS, rnn_hidden_size=64, nb_layers=3,
                       audio_conf=CONF, bidirectional=True)
    pairs = _ds2_pairs(m)
    assert len(pairs) == 3
    before = [p.detach().clone() for p in m.parameters()]
    params = list(m.parameters())
    flat = FlatParams(params, "cpu", adjacent=pairs)
    for p, b in zip(m.parameters(), before):
        assert torch.equal(p.detach(), b)
    flat.zero_grad()                   # as the Trainer before each backward
    for a, b in pairs:
        st = ops._stacked_rows(a, b)
        assert st is not None and torch.equal(st, torch.cat([a, b]))
        ga, gb = ops.grad_like(a), ops.grad_like(b)
        gs = ops._stacked_rows(ga, gb)
        assert gs is not None
        gs.fill_(1.5)
        assert (flat.grad[flat.offset_of[id(a)]:flat.offset_of[id(b)] + b.numel()] == 1.5).all()
    rest = [p for p in reversed(params) if all(p is not a and p is not b for a, b in pairs)]
    order = [p for p in flat.params if all(p is not a and p is not b for a, b in pairs)]
    assert [id(p) for p in order] == [id(p) for p in rest]
    opt = FusedSGD(flat, lr=0.1)
    assert [id(p) for p, _ in opt._model_order()] == [id(p) for p in params]
    # unpaired tensors are not stacked
    assert ops._stacked_rows(params[0], params[1]) is None


def _status_worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ds2amd.optim import global_status_word
    w = torch.zeros(1, dtype=torch.int32)
    if rank == 1:
        w.fill_(1)                 # this rank's recurrence timed out (RNN_ERR_HANDOFF_TIMEOUT)
    global_status_word(w)
    out_q.put((rank, int(w.item())))
    dist.destroy_process_group()


def test_skip_decision_is_global():
    """a hand-off failure on ONE rank must skip the SGD step on EVERY rank (its
    NaN gradients were already all-reduced into every rank's buckets) and make every rank
    raise: the Trainer makes its status word global (MAX over the ranks) before the step.
    gloo world 2, the word set on rank 1 only -> both ranks see it."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_status_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [(0, 1), (1, 1)]


def _fold_worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = _model()
    flat = FlatParams(list(m.parameters()), "cpu", tail=2)
    red = GradAllReducer(flat, bucket_mb=0.0005)
    word = torch.zeros(1, dtype=torch.int32)
    state = {}

    def pack(tail):
        tail[0:1].copy_(word)
        tail[1:2].copy_(state["loss"])

    red.set_status_packer(pack)
    x, y = _data()
    xs, ys = x[rank::world], y[rank::world]
    out = []
    for step in range(2):
        word.fill_(1 if (rank == 1 and step == 1) else 0)   # rank 1 fails in step 1
        flat.zero_grad()
        red.begin()
        loss = ((m(xs) - ys) ** 2).sum(1).mean()
        state["loss"] = loss.detach().reshape(1)
        loss.backward()
        red.finish()
        skip = int(flat.tail[0:1].view(torch.int32).item())
        out.append((float(loss), float(flat.tail[1]), skip, red.collectives, len(red.buckets),
                    red.buckets[-1][1], flat.numel, flat.tail_alloc))
    out_q.put((rank, out))
    dist.destroy_process_group()


def test_status_and_loss_ride_in_the_last_bucket():
    """the step's status word and loss travel in the last gradient bucket's tail
    (FlatParams(tail=2)), so a step issues exactly one collective per bucket -- no separate
    MAX all-reduce of the status word, no reduce_tensor of the loss.  gloo world 2: the tail
    holds the mean loss (data/utils.py:40-44), and a status word set on rank 1 alone makes the
    skip flag non-zero on both ranks (every rank skips, every rank raises)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fold_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for step in range(2):
        losses = [res[r][step][0] for r in range(world)]
        for r in range(world):
            loss, mean, skip, colls, nb, end, numel, tail_alloc = res[r][step]
            assert colls == nb, "one collective per bucket, none for status or loss"
            assert end == numel + tail_alloc, "the last bucket covers the tail"
            assert mean == pytest.approx(sum(losses) / world, rel=1e-6)
            assert (skip != 0) == (step == 1), (r, step, skip)


def test_rccl_cap_defaults(monkeypatch):
    """The guard's CTA budget: NCCL_MAX_NCHANNELS when set (init_distributed sets 32 before the
    communicator exists); unknown when nobody capped RCCL, so the guard always
    waits for the buckets in flight."""
    from ds2amd.optim import rccl_channel_cap, UNKNOWN_CTAS
    monkeypatch.delenv("NCCL_MAX_NCHANNELS", raising=False)
    assert rccl_channel_cap() == UNKNOWN_CTAS
    monkeypatch.setenv("NCCL_MAX_NCHANNELS", "32")
    assert rccl_channel_cap() == 32
    monkeypatch.setenv("NCCL_MAX_NCHANNELS", "junk")
    assert rccl_channel_cap() == UNKNOWN_CTAS
