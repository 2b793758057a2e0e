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
