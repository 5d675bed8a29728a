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
