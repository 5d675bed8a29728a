"""Data-parallel training over RCCL (torch.distributed "nccl" backend == RCCL on ROCm).

One process per GPU. Samples are independent in PerformanceNet (InstanceNorm is per sample,
no BatchNorm), so the only exchange is the gradient all-reduce. Gradients live
in the model's flat buffer (model.flat_buffers), so the all-reduce is a few large bucketed
collectives over contiguous slices — no gradient copies, no per-parameter calls. The mean
over ranks matches one large-batch step: L1 is a mean, so averaging per-rank gradients of
per-rank means equals the gradient of the global mean for equal per-rank batches.
"""
import os

import torch
import torch.distributed as dist

DEFAULT_BUCKET_BYTES = 256 << 20  # 256 MB: big buckets suit xGMI point-to-point rings
# smaller when overlapped: the last bucket is the exposed one (MST_BUCKET_MB: A/B knob)
OVERLAP_BUCKET_BYTES = int(os.environ.get("MST_BUCKET_MB", "128")) << 20
# backward Adam's own buckets when no DP reducer is attached (N = 1; with a reducer it shares the
# reducer's): 64 MB ran the step 0.5 % faster than 128 MB, 32 and 256 MB in between
# (profiles/r05/ab_step_bucket_mb.jsonl; MST_ADAM_BUCKET_MB: A/B knob)
ADAM_BUCKET_BYTES = int(os.environ.get("MST_ADAM_BUCKET_MB", "64")) << 20


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
    op = dist.ReduceOp.AVG if native_avg() else dist.ReduceOp.SUM
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


def flat_buckets(model, bucket_bytes):
    """Cut the model's flat buffers into contiguous buckets of >= bucket_bytes at parameter
    boundaries, in layout order (= the order backward finishes gradients).

    Returns (buckets: [start, end) element ranges covering [0, n), bucket_of: id(param) ->
    bucket index, count: parameters per bucket)."""
    _, _, n = model.flat_buffers()
    f = model._flat
    params = model._flat_params_list()
    spans = sorted((f["index"][id(p)][0], f["index"][id(p)][1], id(p)) for p in params)
    per = max(1, bucket_bytes // 4)
    buckets, bucket_of, count = [], {}, []
    start = 0
    members = []
    for i, (o, k, pid) in enumerate(spans):
        members.append(pid)
        last = i == len(spans) - 1
        end = n if last else spans[i + 1][0]
        if end - start >= per or last:
            b = len(buckets)
            buckets.append((start, end))
            count.append(len(members))
            for q in members:
                bucket_of[q] = b
            members = []
            start = end
    return buckets, bucket_of, count


def native_avg():
    """True when the backend averages inside the collective (ReduceOp.AVG: nccl = RCCL). Other
    backends (gloo) SUM and each bucket is then scaled by 1/world on the stream that waits for
    it, so both paths deliver an averaged bucket at the same point of the stream order."""
    return dist.get_backend() == "nccl"


class OverlappedAllReduce:
    """Gradient all-reduce overlapped with the backward pass.

    The model's flat gradient buffer is laid out in the order backward produces gradients
    (engine.backward_param_order), so it is cut into contiguous buckets at parameter
    boundaries that complete front to back. The backward program reports finished blocks
    (GradSink.block_done -> ready); as soon as every parameter of the next bucket is done, its
    all-reduce is issued from the compute stream (RCCL's stream waits for the gradient
    kernels already enqueued, later backward kernels keep running beside it). Buckets are
    issued strictly in order, so every rank issues the same collectives in the same order.

    `wait_bucket(b)` makes the current stream wait for bucket b's average (BackwardAdam calls it
    on its side stream); `finish()` (Adam.step or dp.finish_gradients) does it for every bucket
    on the compute stream. Gradient accumulation: a new backward pass first finishes the
    previous pass's exchange, so the accumulated buffer holds avg(g1) + g2_local, identical on
    every rank in its first part, and its average is avg(g1) + avg(g2).
    """

    def __init__(self, model, bucket_bytes=OVERLAP_BUCKET_BYTES):
        self.model = model
        _, grad, _ = model.flat_buffers()
        self.buckets, self.bucket_of, self.count = flat_buckets(model, bucket_bytes)
        self.grad = grad
        self.works = []
        self.scaled = []
        self.remaining = list(self.count)
        self.next = 0
        self.active = False

    def begin(self):
        if self.active:
            self.finish()
        self.remaining = list(self.count)
        self.next = 0
        self.works = []
        self.scaled = []
        self.active = is_dist()

    def _launch(self, b):
        s, e = self.buckets[b]
        op = dist.ReduceOp.AVG if native_avg() else dist.ReduceOp.SUM
        self.works.append(dist.all_reduce(self.grad[s:e], op=op, async_op=True))
        self.scaled.append(native_avg())

    def wait_bucket(self, b):
        """The current stream waits for bucket b's averaged gradients."""
        self.works[b].wait()
        if not self.scaled[b]:
            s, e = self.buckets[b]
            self.grad[s:e].mul_(1.0 / dist.get_world_size())
            self.scaled[b] = True

    def ready(self, params):
        if not self.active:
            return
        for p in params:
            b = self.bucket_of.get(id(p))
            if b is not None:
                self.remaining[b] -= 1
        while self.next < len(self.buckets) and self.remaining[self.next] <= 0:
            self._launch(self.next)
            self.next += 1

    def launch_remaining(self):
        if not self.active:
            return
        while self.next < len(self.buckets):
            self._launch(self.next)
            self.next += 1

    def finish(self):
        if not self.active:
            return
        self.launch_remaining()
        for b in range(len(self.works)):
            self.wait_bucket(b)
        self.works = []
        self.active = False


def enable_overlapped_allreduce(model, bucket_bytes=OVERLAP_BUCKET_BYTES):
    """Attach an OverlappedAllReduce to `model`: every backward then all-reduces (averages)
    the gradients while it runs. The package's Adam waits for it; with another optimizer call
    finish_gradients(model) between loss.backward() and optimizer.step()."""
    model._mst_dp = OverlappedAllReduce(model, bucket_bytes)
    return model._mst_dp


def finish_gradients(model):
    r = getattr(model, "_mst_dp", None)
    if r is not None:
        r.finish()
