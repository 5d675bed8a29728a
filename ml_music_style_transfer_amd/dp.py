"""Data-parallel training over RCCL (torch.distributed "nccl" backend == RCCL on ROCm).

One process per GPU. Samples are independent in PerformanceNet (InstanceNorm is per sample,
no BatchNorm), so the only exchange is the gradient all-reduce. Gradients live
in the model's flat buffer (model.flat_buffers), so the all-reduce is a few large bucketed
collectives over contiguous slices — no gradient copies, no per-parameter calls. The mean
over ranks matches one large-batch step: L1 is a mean, so averaging per-rank gradients of
per-rank means equals the gradient of the global mean for equal per-rank batches.
"""
import torch
import torch.distributed as dist

DEFAULT_BUCKET_BYTES = 256 << 20  # 256 MB: big buckets suit xGMI point-to-point rings


def is_dist():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def broadcast_parameters(model, src=0):
    """Make every rank start from rank `src`'s weights (one collective on the flat buffer)."""
    if not is_dist():
        return
    flat, _, n = model.flat_buffers()
    dist.broadcast(flat[:n], src)


def allreduce_gradients(model, bucket_bytes=DEFAULT_BUCKET_BYTES, async_op=False):
    """Average the flat gradient buffer across ranks in contiguous buckets.

    Returns the list of work handles when async_op (caller waits before optimizer.step)."""
    if not is_dist():
        return []
    _, grad, n = model.flat_buffers()
    world = dist.get_world_size()
    per = max(1, bucket_bytes // 4)
    works = []
    op = dist.ReduceOp.AVG if dist.get_backend() == "nccl" else dist.ReduceOp.SUM
    for s in range(0, n, per):
        w = dist.all_reduce(grad[s:min(n, s + per)], op=op, async_op=async_op)
        if async_op:
            works.append(w)
    if op == dist.ReduceOp.SUM:
        for w in works:
            w.wait()
        works = []
        grad[:n].mul_(1.0 / world)
    return works


def wait_all(works):
    for w in works:
        w.wait()
