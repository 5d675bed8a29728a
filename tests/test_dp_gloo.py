"""Data-parallel path (ml_music_style_transfer_amd.dp) on CPU with gloo, world_size 2.

The GPU path uses the same functions over RCCL ("nccl"); here the flat buffers are CPU
tensors of a stand-in model. Also checks the math the DP design relies on: with a per-rank
mean loss (L1, train.py:132) and equal per-rank batches, the average of per-rank gradients is
the full-batch gradient (oracle/model_ref.py on a small PerformanceNet-shaped problem).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class _FlatModel:
    def __init__(self, n, rank):
        g = torch.Generator().manual_seed(100 + rank)
        self.param = torch.randn(n, generator=g)
        self.grad = torch.randn(n, generator=g)

    def flat_buffers(self):
        return self.param, self.grad, self.param.numel()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, bucket, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ml_music_style_transfer_amd import dp
    m = _FlatModel(n, rank)
    dp.broadcast_parameters(m)
    works = dp.allreduce_gradients(m, bucket_bytes=bucket)
    dp.wait_all(works)
    q.put((rank, m.param.clone(), m.grad.clone()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n,bucket", [(1000, 4 * 128), (4099, 1 << 20)])
def test_allreduce_and_broadcast_gloo(n, bucket):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, bucket, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (pp, gg)) for r, pp, gg in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = [_FlatModel(n, r) for r in range(world)]
    mean_grad = sum(m.grad for m in ref) / world
    for r in range(world):
        torch.testing.assert_close(res[r][0], ref[0].param)         # rank 0's weights everywhere
        torch.testing.assert_close(res[r][1], mean_grad, rtol=1e-6, atol=1e-6)


def test_per_rank_mean_gradients_average_to_full_batch():
    """L1 is a mean, so (g_rank0 + g_rank1)/2 == gradient of the full batch."""
    torch.manual_seed(0)
    W = torch.randn(6, 5, 3, dtype=torch.float64, requires_grad=True)
    x = torch.randn(4, 5, 12, dtype=torch.float64)
    t = torch.randn(4, 6, 12, dtype=torch.float64)

    def grad(xb, tb):
        W.grad = None
        y = torch.nn.functional.conv1d(xb, W, padding=1)
        torch.nn.functional.instance_norm(y).sub(tb).abs().mean().backward()
        return W.grad.clone()

    full = grad(x, t)
    halves = (grad(x[:2], t[:2]) + grad(x[2:], t[2:])) / 2
    torch.testing.assert_close(halves, full)


class _LayeredModel:
    """Stand-in exposing what OverlappedAllReduce uses of PerformanceNet's flat buffers."""

    def __init__(self, sizes, rank):
        self.params = [torch.nn.Parameter(torch.empty(k)) for k in sizes]
        offs, off = [], 0
        for k in sizes:
            offs.append(off)
            off += (k + 3) // 4 * 4
        self.flat = torch.zeros(off)
        self.gradbuf = torch.zeros(off)
        g = torch.Generator().manual_seed(7 + rank)
        for p, o in zip(self.params, offs):
            self.gradbuf[o:o + p.numel()] = torch.randn(p.numel(), generator=g)
        self._flat = {"index": {id(p): (o, p.numel()) for p, o in zip(self.params, offs)}}
        self.n = off

    def flat_buffers(self):
        return self.flat, self.gradbuf, self.n

    def _flat_params_list(self):
        return self.params


def _overlap_worker(rank, world, port, sizes, bucket, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ml_music_style_transfer_amd import dp
    m = _LayeredModel(sizes, rank)
    r = dp.OverlappedAllReduce(m, bucket_bytes=bucket)
    r.begin()
    launched = []
    for i in range(0, len(m.params), 2):   # "blocks" of two parameters finish in layout order
        r.ready(m.params[i:i + 2])
        launched.append(r.next)
    r.finish()
    q.put((rank, m.gradbuf.clone(), len(r.buckets), launched))
    dist.barrier()
    dist.destroy_process_group()


def test_overlapped_bucket_allreduce_gloo():
    """Buckets are issued as soon as their parameters are done, in order, and the result is
    the rank average (dp.OverlappedAllReduce, the path bench.py uses for N > 1)."""
    sizes = [5, 17, 3, 64, 9, 1, 33, 8]
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, world, port, sizes, 4 * 24, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (g, nb, la)) for r, g, nb, la in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    mean = sum(_LayeredModel(sizes, r).gradbuf for r in range(world)) / world
    for r in range(world):
        g, nb, launched = res[r]
        assert nb > 2
        assert launched == sorted(launched) and launched[0] >= 1  # issued during "backward"
        torch.testing.assert_close(g, mean, rtol=1e-6, atol=1e-6)


def _native_avg_worker(rank, world, port, sizes, bucket, q):
    """The RCCL-only branches (dp.native_avg() True: ReduceOp.AVG issued, no SUM-then-scale in
    wait_bucket / allreduce_gradients) over gloo through tests/_rccl_emulation.py."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import _rccl_emulation
    dp = _rccl_emulation.install()
    m = _LayeredModel(sizes, rank)
    r = dp.OverlappedAllReduce(m, bucket_bytes=bucket)
    r.begin()
    for i in range(0, len(m.params), 2):
        r.ready(m.params[i:i + 2])
    native = all(r.scaled)          # every issued bucket took the AVG branch
    r.finish()
    over = m.gradbuf.clone()
    m2 = _LayeredModel(sizes, rank)
    dp.wait_all(dp.allreduce_gradients(m2, bucket_bytes=bucket, async_op=True))
    q.put((rank, native, over, m2.gradbuf.clone()))
    dist.barrier()
    dist.destroy_process_group()


def test_native_avg_branches_emulated_gloo():
    """OverlappedAllReduce._launch / wait_bucket and allreduce_gradients on the path RCCL takes
    (ReduceOp.AVG, no host-side scale): equal to the rank mean, and bitwise equal between the
    overlapped and the post-backward forms."""
    sizes = [5, 17, 3, 64, 9, 1, 33, 8]
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_native_avg_worker, args=(r, world, port, sizes, 4 * 24, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    mean = sum(_LayeredModel(sizes, r).gradbuf for r in range(world)) / world
    for r in range(world):
        native, over, post = res[r]
        assert native
        torch.testing.assert_close(over, mean, rtol=1e-6, atol=1e-6)
        assert torch.equal(over, post)
