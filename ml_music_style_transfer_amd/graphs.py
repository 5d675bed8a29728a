"""hipGraph capture of the PerformanceNet programs (torch.cuda.CUDAGraph records a hipGraph).

The eager forward is ~150 kernel launches issued from Python through ctypes; at the
inference batch (B = 1, one 4-second chunk, inference.py:74-91) the GPU work per launch is
tens of microseconds, so eager inference is host-bound. A captured graph replays the same
kernels with one launch from the host.

GraphedForward     eval forward at a fixed input shape (AudioSynthesizer's model call).
GraphedTrainStep   forward + nn.L1Loss + backward + Adam (train.py:131-141) at a fixed batch
                   shape, one replay per step. The step-dependent values live on the device:
                   the dropout seed counter (mst_conv_desc.seed_dev) and Adam's bias-correction
                   pair (mst_adam_dev_f32), both advanced by the graph itself, so every replay
                   is a fresh step (new dropout masks, next step count); the learning rate is a
                   device scalar refreshed before a replay when the group's lr changed.

Both copy their inputs into static device buffers and return static outputs (overwritten by
the next call: clone what must be kept). Single GPU; the data-parallel step keeps the eager
overlapped all-reduce (dp.py).
"""
import math

import torch

from . import kernels as K
from . import ops as _ops  # noqa: F401  (registers torch.ops.mst.*)

# odd 64-bit stride of the device dropout-seed counter: successive steps key far-apart seeds
SEED_STRIDE = 0x9E3779B97F4A7C15 & 0x7FFFFFFFFFFFFFFF


def _static_like(t):
    return torch.empty(t.shape, device=t.device, dtype=torch.float32)


class GraphedForward:
    """model(x_midi, x_audio, cond) in eval mode / no_grad, captured once for this shape."""

    def __init__(self, model, x_midi, x_audio, cond, warmup=2):
        if not torch.cuda.is_available():
            raise RuntimeError("GraphedForward needs a HIP device")
        self.model = model.eval()
        self.inputs = [_static_like(t) for t in (x_midi, x_audio, cond)]
        for s, t in zip(self.inputs, (x_midi, x_audio, cond)):
            s.copy_(t)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side), torch.no_grad():
            for _ in range(warmup):  # sizes the workspace arena and the allocator pools
                self.model(*self.inputs)
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(self.graph):
            self.out = self.model(*self.inputs)

    def __call__(self, x_midi, x_audio, cond):
        for s, t in zip(self.inputs, (x_midi, x_audio, cond)):
            s.copy_(t, non_blocking=True)
        self.graph.replay()
        return self.out


class GraphedTrainStep:
    """One Adam training step of a flat-buffer PerformanceNet on (x_midi, x_audio, cond,
    target), captured after `warmup` eager steps of the same program. Every call is one real
    training step (the warmup calls included). Requires train.Adam with one parameter group
    over the model's flat parameters, no overlapped-backward or data-parallel hooks."""

    def __init__(self, model, optimizer, warmup=2):
        if not torch.cuda.is_available():
            raise RuntimeError("GraphedTrainStep needs a HIP device")
        if getattr(model, "_mst_dp", None) is not None or getattr(model, "_mst_adam", None) is not None:
            raise ValueError("GraphedTrainStep: detach the data-parallel / backward-Adam hooks")
        if len(optimizer.param_groups) != 1:
            raise ValueError("GraphedTrainStep: one parameter group over the flat parameters")
        self.model, self.opt = model, optimizer
        pf, gf, n = model.flat_buffers()
        index = model._flat["index"]
        self.params = [p for p in optimizer.param_groups[0]["params"] if id(p) in index]
        if len(self.params) != len(index):
            raise ValueError("GraphedTrainStep: the group must hold every flat parameter")
        self.pf, self.gf = pf, gf
        dev = pf.device
        self.warmup = warmup
        self.calls = 0
        self.graph = None
        self._captured_st = None  # the flat Adam state whose m/v buffers the graph names
        self.inputs = None
        g = optimizer.param_groups[0]
        self.b1, self.b2 = g["betas"]
        self.eps = g["eps"]
        # device state advanced by the program itself
        self.seed_dev = torch.zeros((), device=dev, dtype=torch.int64)
        model.__dict__["_mst_seed_dev"] = self.seed_dev
        self.step_dev = None  # float64 step count, built with the flat Adam state
        self._host_step = None
        self.lr_dev = torch.full((), float(g["lr"]), device=dev, dtype=torch.float64)
        self._lr = float(g["lr"])
        self.hyper = torch.zeros(2, device=dev, dtype=torch.float32)
        self.loss = torch.zeros((), device=dev, dtype=torch.float32)

    def _state(self):
        st = self.opt._flat_state(0, self.pf, self.params)
        if st is None:
            raise ValueError("GraphedTrainStep: parameters have differing Adam step counts")
        if self.step_dev is None:
            self.step_dev = torch.full((), float(st["step"]), device=self.pf.device,
                                       dtype=torch.float64)
        elif st["step"] != self._host_step:  # eager optimizer steps ran in between
            self.step_dev.fill_(float(st["step"]))
        self._host_step = st["step"]
        if self.graph is not None and st is not self._captured_st:
            # the optimizer rebuilt its flat moments (load_state_dict): the captured graph
            # still names the old m/v buffers, so capture again over the new ones
            self.graph = None
        return st

    def _program(self, st):
        """The step as device work only (no host reads), eager or under capture."""
        m = self.model
        self.seed_dev.add_(SEED_STRIDE)
        self.step_dev.add_(1.0)
        bc1 = 1.0 - torch.pow(self.b1, self.step_dev)
        bc2 = 1.0 - torch.pow(self.b2, self.step_dev)
        self.hyper.copy_(torch.stack((self.lr_dev / bc1, torch.sqrt(bc2))))
        for p in self.params:
            p.grad = None  # the backward program writes (not accumulates) into the flat slots
        y = m(*self.inputs[:3])
        loss = torch.ops.mst.l1_loss(y, self.inputs[3])
        loss.backward()
        K.adam_dev(self.pf, self.gf, st["m"], st["v"], self.hyper, self.b1, self.b2, self.eps)
        self.loss.copy_(loss)

    def __call__(self, x_midi, x_audio, cond, target):
        srcs = (x_midi, x_audio, cond, target)
        if self.inputs is None:
            self.inputs = [_static_like(t) for t in srcs]
        for s, t in zip(self.inputs, srcs):
            if s.shape != t.shape:
                raise ValueError("GraphedTrainStep: input shapes are fixed at first call")
            s.copy_(t, non_blocking=True)
        lr = float(self.opt.param_groups[0]["lr"])
        if lr != self._lr:
            self.lr_dev.fill_(lr)
            self._lr = lr
        st = self._state()
        self.model.train()
        if self.graph is not None:
            self.graph.replay()
        elif self.calls < self.warmup:
            self._program(st)
        else:
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self._program(st)
            self._captured_st = st
            self.graph.replay()
        self.calls += 1
        self.opt._count_step(st, self.params)
        self._host_step = st["step"]
        return self.loss


def inference_step_times(model, B=1, T=252, iters=20, warmup=3):
    """(eager host ms per forward, eager device ms, graphed device ms) at (B, T): the host time
    is the wall time of issuing one eager forward; if it exceeds the device time the eager
    path is host-bound, and the graphed replay time is what the device needs."""
    import time
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    xm = (torch.rand(B, 128, T, generator=g) > 0.9).float().to(dev)
    xa = torch.rand(B, 1025, T, generator=g).to(dev)
    cd = (torch.rand(B, 128, T, generator=g) > 0.95).float().to(dev)
    model.eval()
    with torch.no_grad():
        for _ in range(warmup):
            model(xm, xa, cd)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            model(xm, xa, cd)
        t_issue = (time.perf_counter() - t0) * 1e3 / iters
        e1.record()
        torch.cuda.synchronize()
        eager_dev = e0.elapsed_time(e1) / iters
    gf = GraphedForward(model, xm, xa, cd)
    for _ in range(warmup):
        gf(xm, xa, cd)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        gf(xm, xa, cd)
    e1.record()
    torch.cuda.synchronize()
    graphed = e0.elapsed_time(e1) / iters
    return {"B": B, "T": T, "eager_host_issue_ms": t_issue, "eager_wall_ms": eager_dev,
            "graphed_ms": graphed, "host_bound_eager": t_issue > graphed,
            "speedup": eager_dev / graphed if graphed > 0 else math.nan}
