"""Drop-in for the reference training step API (model/train.py).

`train(model, epoch, train_loader, optimizer, iter_train_loss)` and
`test(model, epoch, test_loader, scheduler, iter_test_loss)` keep the
reference's signatures, loop structure, prints and return values
(train.py:125-170); the loss is the device L1 (engine.l1_loss) and `Adam`
is a torch.optim.Optimizer whose step runs one fused kernel over the model's
flat parameter buffer (torch.optim.Adam semantics, state_dict format included,
so ReduceLROnPlateau and checkpointing work unchanged).

The HDF5 data path (Dataseth5py / Process_Data, train.py:45-116) is in data.py
(libhdf5 through ctypes; h5py is absent). `SyntheticSpectrogramDataset` produces
batches of the same (data (B,256,T), data_cond (B,1025,T), target (B,1025,T))
shape when no HDF5 files are given.
"""
import argparse
import json
import math
import os

import numpy as np
import torch

from . import dp
from . import engine as E
from . import kernels as K
from .model import PerformanceNet, slot_view


class hyperparams(object):
    """train.py:32-42."""

    def __init__(self, args):
        self.train_epoch = args.epochs
        self.test_freq = args.test_freq
        self.exp_name = args.exp_name
        self.iter_train_loss = []
        self.iter_test_loss = []
        self.loss_history = []
        self.test_loss_history = []
        self.best_loss = 1e10
        self.best_epoch = 0


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam (no weight decay / amsgrad) with a fused device update.

    When every parameter of a group with a gradient lives in one PerformanceNet flat
    buffer (and its gradient in the matching flat gradient buffer) the update is one
    kernel launch over the whole buffer; otherwise one launch per parameter.
    """

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0,
                 amsgrad=False):
        if weight_decay != 0 or amsgrad:
            raise NotImplementedError("the reference uses Adam(lr=1e-3) only (train.py:188)")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=0, amsgrad=False))
        self._flat_groups = {}

    def _flat_of(self, group, params):
        """Return (flat_param, flat_grad, numel, offsets) if params tile one model's flat buffers."""
        ref = getattr(params[0], "_mst_flat_owner", None)
        owner = ref() if ref is not None else getattr(self, "_owner", None)
        if owner is None or not owner._flat_ok():
            return None
        self._owner = owner
        pf, gf, n = owner.flat_buffers()
        index = owner._flat["index"]
        if len(params) != len(index):
            return None
        base_p, base_g = pf.data_ptr(), gf.data_ptr()
        for p in params:
            ent = index.get(id(p))
            if ent is None or p.grad is None:
                return None
            o = ent[0]
            if p.data_ptr() != base_p + 4 * o or p.grad.data_ptr() != base_g + 4 * o:
                return None
        return pf, gf, n

    def attach(self, model):
        """Declare the PerformanceNet whose flat buffers the parameters live in."""
        self._owner = model
        return self

    def overlap_backward(self, model=None, bucket_bytes=dp.ADAM_BUCKET_BYTES):
        """Run this optimizer's update inside the model's backward pass, bucket by bucket
        (BackwardAdam). Only for loops that call step() after every backward (the reference's
        train loop, train.py:131-141): no gradient accumulation across backward passes, no
        gradient inspection or clipping between backward and step."""
        if model is not None:
            self._owner = model
        self._bwd = BackwardAdam(self, self._owner, bucket_bytes)
        self._owner._mst_adam = self._bwd
        return self

    def _flat_state(self, gi, pf, params):
        """Flat m/v buffers (and the shared step count) of a flat-buffer group, built on first
        use. Moments already in self.state (load_state_dict, or earlier per-parameter steps)
        are copied into the flat slots. None when the parameters' step counts differ: the
        per-parameter path then keeps torch's per-parameter bias correction."""
        key = (gi, pf.data_ptr())
        st = self._flat_groups.get(key)
        if st is None:
            steps = {float(self.state[p]["step"]) for p in params
                     if self.state.get(p, {}).get("exp_avg") is not None}
            if len(steps) > 1 or (steps and any(
                    self.state.get(p, {}).get("exp_avg") is None for p in params)):
                return None
            m = torch.zeros_like(pf)
            v = torch.zeros_like(pf)
            st = {"m": m, "v": v, "step": int(steps.pop()) if steps else 0}
            index = self._owner._flat["index"]
            for p in params:
                o, k = index[id(p)]
                mv, vv = slot_view(m[o:o + k], p), slot_view(v[o:o + k], p)
                old = self.state.get(p, {})
                if old.get("exp_avg") is not None:
                    mv.copy_(old["exp_avg"])
                    vv.copy_(old["exp_avg_sq"])
                self.state[p] = {"step": torch.tensor(float(st["step"])), "exp_avg": mv,
                                 "exp_avg_sq": vv}
            self._flat_groups[key] = st
        return st

    def prepare(self):
        """Allocate the flat moment buffers now instead of at the first step (same values: zeros,
        or the loaded per-parameter moments). Returns self."""
        owner = getattr(self, "_owner", None)
        if owner is None or not owner._flat_ok():
            return self
        index = owner._flat["index"]
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if id(p) in index]
            flat = self._flat_of(group, params) if params else None
            if flat is not None:
                self._flat_state(gi, flat[0], params)
        return self

    def load_state_dict(self, state_dict):
        """torch.optim.Optimizer.load_state_dict; the flat moment buffers are rebuilt from the
        loaded per-parameter state on the next step (resume keeps exp_avg/exp_avg_sq/step)."""
        super().load_state_dict(state_dict)
        self._flat_groups = {}

    def _count_step(self, st, params):
        st["step"] += 1
        for p in params:  # one tensor per parameter: the per-parameter path adds in place
            self.state[p]["step"] = torch.tensor(float(st["step"]))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        owner = getattr(self, "_owner", None)
        reducer = getattr(owner, "_mst_dp", None) if owner is not None else None
        if reducer is not None:
            reducer.finish()  # overlapped data-parallel all-reduce must land first
        bwd = getattr(self, "_bwd", None)
        if bwd is not None and bwd.finish():  # the update already ran inside backward
            self._count_step(bwd.st, bwd.params)
            return loss
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            lr, eps = group["lr"], group["eps"]
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            flat = self._flat_of(group, params)
            st = self._flat_state(gi, flat[0], params) if flat is not None else None
            if st is not None:
                pf, gf, n = flat
                t = st["step"] + 1
                bc1 = 1 - b1 ** t
                bc2 = 1 - b2 ** t
                K.adam(pf, gf, st["m"], st["v"], lr / bc1, b1, b2, eps, math.sqrt(bc2))
                self._count_step(st, params)
                continue
            for p in params:
                state = self.state[p]
                if len(state) == 0 or state.get("exp_avg") is None:
                    state["step"] = torch.tensor(0.0)
                    state["exp_avg"] = torch.zeros_like(p)  # p's strides (tap-major slots too)
                    state["exp_avg_sq"] = torch.zeros_like(p)
                state["step"] += 1
                t = float(state["step"])
                bc1 = 1 - b1 ** t
                bc2 = 1 - b2 ** t
                _adam_param(p, state, lr / bc1, b1, b2, eps, math.sqrt(bc2))
        return loss


def _memory_order(t):
    """Dimension permutation that lists t's dims from the largest stride to the smallest: for a
    dense tensor, t.permute(perm) is contiguous (a tap-major slot view (d0, d1, k) of (d0, k, d1)
    memory gives perm (0, 2, 1))."""
    return sorted(range(t.dim()), key=lambda d: (-t.stride(d), d))


def _adam_param(p, state, lr_step, b1, b2, eps, bc2_sqrt):
    """One parameter's update. adam_kernel walks raw memory, so p, its gradient and both
    moments are handed over in p's memory order: the gradient (any layout) is permuted into it,
    the moments are re-laid-out to p's strides once if they differ (e.g. loaded from a
    checkpoint), and a non-dense p is updated through a contiguous copy."""
    for key in ("exp_avg", "exp_avg_sq"):
        x = state[key]
        if x.stride() != p.stride():
            y = torch.empty_like(p)
            y.copy_(x)
            state[key] = y
    perm = _memory_order(p)
    pv = p.data.permute(perm)
    mv, vv = state["exp_avg"].permute(perm), state["exp_avg_sq"].permute(perm)
    g = p.grad.permute(perm).contiguous()
    if pv.is_contiguous() and mv.is_contiguous() and vv.is_contiguous():
        K.adam(pv, g, mv, vv, lr_step, b1, b2, eps, bc2_sqrt)
        return
    pc, mc, vc = pv.contiguous(), mv.contiguous(), vv.contiguous()
    K.adam(pc, g, mc, vc, lr_step, b1, b2, eps, bc2_sqrt)
    pv.copy_(pc)
    mv.copy_(mc)
    vv.copy_(vc)


class BackwardAdam:
    """Adam updates issued inside the backward pass, one flat-buffer bucket at a time, on a side
    stream (Adam.overlap_backward).

    The flat buffers are laid out in the order backward finishes with each parameter
    (engine.backward_param_order), and the backward program reports a block done only after
    the block's last read of its weights (its input-gradient GEMM). A bucket whose parameters
    are all done is final: its update (adam_kernel over the bucket's range: per element the
    same arithmetic as one launch over the whole buffer) goes to a second stream that waits for
    the compute stream at that point, so the HBM-bound update runs beside the MFMA-bound
    backward GEMMs. With the data-parallel reducer attached a bucket's update waits for that
    bucket's RCCL all-reduce instead. step() then joins the side stream and counts the step.

    Inactive (step() runs the ordinary update) unless one parameter group holds exactly the
    model's flat parameters, and when gradients are reduced after backward (world > 1 without
    an overlapped reducer). Any backend works: with gloo the reducer's per-bucket SUM is scaled
    to the average on this side stream before the update (dp.OverlappedAllReduce.wait_bucket)."""

    def __init__(self, opt, model, bucket_bytes):
        self.opt = opt
        self.model = model
        reducer = getattr(model, "_mst_dp", None)
        if reducer is not None:
            self.buckets, self.bucket_of, self.count = reducer.buckets, reducer.bucket_of, reducer.count
        else:
            self.buckets, self.bucket_of, self.count = dp.flat_buckets(model, bucket_bytes)
        pf, _, _ = model.flat_buffers()
        self.stream = torch.cuda.Stream(device=pf.device)
        self.active = self.launched = False
        self.st = self.params = None
        self.updates = 0  # steps whose update ran inside backward
        self.joined = None  # event of the last finish(): completes with that step's updates
        self.max_blocks = int(os.environ.get("MST_BWD_ADAM_BLOCKS", "256"))  # A/B tuning knob
        self.paused = False  # True: step() runs the one-launch update (bench.py's GEMM timing leg)

    def _eligible(self):
        m = self.model
        if len(self.opt.param_groups) != 1 or not m._flat_ok():
            return False
        # the group may also hold parameters outside the flat buffer (the dead MBR convolutions,
        # model.py:143-174): backward never gives them a gradient, so Adam skips them anyway
        index = m._flat["index"]
        params = [p for p in self.opt.param_groups[0]["params"] if id(p) in index]
        if len(params) != len(index) or not all(p.requires_grad for p in params):
            return False
        if dp.is_dist():
            reducer = getattr(m, "_mst_dp", None)
            if reducer is None or reducer.buckets is not self.buckets:
                return False
        return True

    def begin(self):
        self.active = self.launched = False
        if self.paused or not self._eligible():
            return
        group = self.opt.param_groups[0]
        index = self.model._flat["index"]
        self.params = [p for p in group["params"] if id(p) in index]
        self.pf, self.gf, _ = self.model.flat_buffers()
        self.st = self.opt._flat_state(0, self.pf, self.params)
        if self.st is None:
            return
        b1, b2 = group["betas"]
        t = self.st["step"] + 1
        self.hp = (group["lr"] / (1 - b1 ** t), b1, b2, group["eps"], math.sqrt(1 - b2 ** t))
        self.remaining = list(self.count)
        self.next = 0
        self.active = True

    def _launch(self, b):
        s, e = self.buckets[b]
        reducer = getattr(self.model, "_mst_dp", None)
        compute = torch.cuda.current_stream()
        with torch.cuda.stream(self.stream):
            if reducer is not None and reducer.active:
                reducer.wait_bucket(b)  # this stream waits for bucket b's averaged gradients
            else:
                self.stream.wait_stream(compute)
            # one workgroup per CU: a background stream beside the backward GEMMs, which keep
            # their two workgroups per CU (a full-width grid would take their slots instead)
            K.adam(self.pf[s:e], self.gf[s:e], self.st["m"][s:e], self.st["v"][s:e], *self.hp,
                   max_blocks=self.max_blocks)

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
        self.launched = True

    def finish(self):
        """Join the side stream. True when this backward's update has been issued."""
        if not (self.active and self.launched):
            return False
        ev = torch.cuda.Event()
        ev.record(self.stream)
        torch.cuda.current_stream().wait_event(ev)
        self.joined = ev  # completes with this step's last bucket update
        self.active = self.launched = False
        self.updates += 1
        return True


def make_optimizer(model, lr=1e-3, overlap_backward=False):
    """optim.Adam(model.parameters(), lr=1e-3) (train.py:188) bound to the model's flat buffers;
    overlap_backward=True runs its update inside backward (BackwardAdam)."""
    opt = Adam(model.parameters(), lr=lr).attach(model)
    return opt.overlap_backward() if overlap_backward else opt


def _cuda(t):
    return t if t.is_cuda else t.cuda(non_blocking=True)


LOSSES = ("l1", "mss", "l1+mss")


def make_loss(name="l1", mss_phase="griffinlim", gl_iters=8, alpha=1.0, sizes=None, hop=256):
    """The training loss, loss_fn(y_pred, target) on (B, 1025, T) log-power spectrograms:
      l1      nn.L1Loss (train.py:132-135), the reference's loss;
      mss     the README's multi-scale spectral loss (README.md:23; the engel_loss stub,
              train.py:119-123) on rendered audio, spectral.spectrogram_mss_loss: the target is
              the Griffin-Lim reconstruction of the target spectrogram (gl_iters iterations; the
              HDF5 data holds no audio), the prediction is rendered with mss_phase's phase
              ("griffinlim": its own reconstruction's, "target": the target reconstruction's);
      l1+mss  their sum.
    The target waveform is a constant of each item: a data.DeviceLoader given
    `loss_fn.target_audio` as its target_audio computes it once per item and hands it over as
    `target.mst_audio`; a target without it (any other loader) is reconstructed per call. Griffin-
    Lim from the same spectrogram is bitwise the same per clip in any batch (spectral.griffinlim),
    so both paths give the same loss."""
    if name not in LOSSES:
        raise ValueError(f"loss {name!r}: one of {LOSSES}")
    from . import spectral

    def target_audio(target):
        with torch.no_grad():
            return spectral.griffinlim(target, n_iter=gl_iters, hop_length=hop, init=None,
                                       from_logpow=True)

    def mss(y_pred, target):
        if y_pred.shape != target.shape:
            raise ValueError("the multi-scale loss needs T = 12 (mod 16) (model.py:229-232)")
        y_t = getattr(target, "mst_audio", None)
        if y_t is None:
            y_t = target_audio(target)
        return spectral.spectrogram_mss_loss(y_pred, y_t, phase=mss_phase, hop=hop, alpha=alpha,
                                             sizes=sizes, gl_iters=gl_iters)

    if name == "l1":
        return E.l1_loss
    fn = mss if name == "mss" else (lambda y_pred, target: E.l1_loss(y_pred, target) + mss(y_pred, target))
    fn.target_audio = target_audio
    return fn


def train(model, epoch, train_loader, optimizer, iter_train_loss, log_every=2, loss_fn=None):
    """train.py:125-149 (same loop, loss and prints); loss_fn defaults to train.py:132's L1
    (make_loss selects the multi-scale spectral loss instead)."""
    model.train()
    train_loss = 0
    loss_fn = loss_fn or E.l1_loss
    for batch_idx, (data, data_cond, target) in enumerate(train_loader):
        optimizer.zero_grad()
        split = torch.split(data, 128, dim=1)
        y_pred = model(_cuda(split[0]), _cuda(data_cond), _cuda(split[1]))
        loss = loss_fn(y_pred, _cuda(target))
        loss.backward()
        dp.finish_gradients(model)  # no-op unless an overlapped DP all-reduce is attached
        iter_train_loss.append(loss.item())
        train_loss += loss
        optimizer.step()
        if log_every and batch_idx % log_every == 0:
            print('Train Epoch: {} [{}/{} ({:.0f}%)]\t Loss: {:.6f}'.format(
                epoch, batch_idx * len(data), len(train_loader.dataset),
                100. * batch_idx / len(train_loader), loss.item() / len(data)))
    train_loss = _sum_over_ranks(train_loss)  # data parallel: every rank's batches
    print('====> Epoch: {} Average loss: {:.4f}'.format(epoch, train_loss / len(train_loader.dataset)))
    return train_loss / len(train_loader.dataset)


def test(model, epoch, test_loader, scheduler, iter_test_loss):
    """train.py:152-170 (MSE on the device, ReduceLROnPlateau step)."""
    with torch.no_grad():
        model.eval()
        test_loss = 0
        for idx, (data, data_cond, target) in enumerate(test_loader):
            split = torch.split(data, 128, dim=1)
            y_pred = model(_cuda(split[0]), _cuda(data_cond), _cuda(split[1]))
            loss = E.mse_loss(y_pred, _cuda(target))
            iter_test_loss.append(loss.item())
            test_loss += loss
        test_loss = _sum_over_ranks(test_loss)  # one scheduler decision on every rank
        test_loss /= len(test_loader.dataset)
        scheduler.step(test_loss)
        print('====> Test set loss: {:.4f}'.format(test_loss))
        return test_loss


class SyntheticSpectrogramDataset(torch.utils.data.Dataset):
    """Stand-in for Dataseth5py (train.py:45-104) with the same item layout:
    X = concat(pianoroll, onoff).T (256, T), X_cond = random same-style spec, y = spec."""

    def __init__(self, n, T=252, seed=0, device="cuda"):
        g = torch.Generator().manual_seed(seed)
        roll = (torch.rand(n, 128, T, generator=g) < 0.08).float()
        prev = torch.cat([torch.zeros(n, 128, 1), roll[:, :, :-1]], 2)
        self.X = torch.cat([roll, roll - prev], 1).to(device)
        self.spec = (torch.rand(n, 1025, T, generator=g) * 2).pow(2).to(device)
        self.rand_index = torch.randint(0, n, (n,), generator=g)
        self.n = n

    def __getitem__(self, i):
        return self.X[i], self.spec[int(self.rand_index[i])], self.spec[i]

    def __len__(self):
        return self.n


def _init_data_parallel():
    """One process per GPU under torch.distributed.run (WORLD_SIZE > 1): backend nccl (= RCCL
    over xGMI), or $MST_DIST_BACKEND (gloo: ranks may share a GPU, for rehearsal/tests)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1
    import torch.distributed as dist
    backend = os.environ.get("MST_DIST_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend != "nccl":
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend)
    return dist.get_rank(), dist.get_world_size()


def _sum_over_ranks(t):
    if dp.is_dist() and isinstance(t, torch.Tensor):
        import torch.distributed as dist
        t = t.detach().clone()
        dist.all_reduce(t)
    return t


def main(args, return_model=False):
    """train.py:173-208. Reads `<data_dir>_train.hdf5` / `_test.hdf5` (data.Process_Data,
    HBM-resident loaders) when they exist, else a synthetic dataset of the same layout."""
    hp = hyperparams(args)
    rank, world = _init_data_parallel()
    exp_root = os.path.join(os.path.abspath('./'), 'experiments')
    os.makedirs(exp_root, exist_ok=True)
    exp_dir = os.path.join(exp_root, hp.exp_name)
    os.makedirs(exp_dir, exist_ok=True)
    model = PerformanceNet().cuda()
    if world > 1:
        dp.broadcast_parameters(model)         # every rank starts from rank 0's weights
        dp.enable_overlapped_allreduce(model)  # bucket all-reduces inside backward
        model._seed += rank << 24              # per-rank dropout streams
    # the reference loop steps after every backward (train.py:131-141), so the update runs per
    # bucket inside backward (BackwardAdam: bitwise the one-launch update, 1.5-2.3 % faster)
    optimizer = make_optimizer(model, lr=1e-3, overlap_backward=True)
    model.zero_grad()
    optimizer.zero_grad()
    scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, 'min')
    loss_fn = make_loss(getattr(args, "loss", "l1"), mss_phase=getattr(args, "mss_phase", "griffinlim"),
                        gl_iters=getattr(args, "gl_iters", 8))
    if args.data_dir and os.path.exists(args.data_dir + '_train.hdf5'):
        from .data import DeviceLoader, Process_Data
        train_loader, test_loader = Process_Data(args.data_dir, n_train_read=args.n_train_read,
                                                 n_test_read=args.n_test_read,
                                                 batch_size=args.batch_size)
        if world > 1:  # one shard of every epoch per rank, per-rank style/cond draws
            from torch.utils.data.distributed import DistributedSampler
            import random
            random.seed(42 + rank)
            tr, te = train_loader.dataset, test_loader.dataset
            train_loader = DeviceLoader(tr, args.batch_size, sampler=DistributedSampler(
                tr, num_replicas=world, rank=rank, shuffle=True))
            test_loader = DeviceLoader(te, args.batch_size, sampler=DistributedSampler(
                te, num_replicas=world, rank=rank, shuffle=False))
        # the multi-scale loss's target waveform: once per item, kept in HBM beside the split
        train_loader.target_audio = getattr(loss_fn, "target_audio", None)
    else:
        T = args.frames
        train_ds = SyntheticSpectrogramDataset(args.n_train_read or 32, T=T, seed=1)
        test_ds = SyntheticSpectrogramDataset(args.n_test_read or 8, T=T, seed=2)
        train_loader = torch.utils.data.DataLoader(train_ds, batch_size=args.batch_size,
                                                   shuffle=True)
        test_loader = torch.utils.data.DataLoader(test_ds, batch_size=args.batch_size)
    print('start training')
    for epoch in range(hp.train_epoch):
        if hasattr(train_loader, "set_epoch"):
            train_loader.set_epoch(epoch)
        loss = train(model, epoch, train_loader, optimizer, hp.iter_train_loss, loss_fn=loss_fn)
        hp.loss_history.append(loss.item())
        if epoch % hp.test_freq == 0:
            test_loss = test(model, epoch, test_loader, scheduler, hp.iter_test_loss)
            hp.test_loss_history.append(test_loss.item())
            if test_loss < hp.best_loss:
                hp.best_loss = test_loss.item()
                hp.best_epoch = epoch + 1
                if rank != 0:
                    continue
                print("saving model")
                torch.save({'epoch': epoch + 1, 'state_dict': model.state_dict(),
                            'optimizer': optimizer.state_dict()},
                           os.path.join(exp_dir, 'checkpoint-{}.tar'.format(str(epoch + 1))))
                with open(os.path.join(exp_dir, 'hyperparams.json'), 'w') as outfile:
                    json.dump(hp.__dict__, outfile)
    return (hp, model) if return_model else hp


def parse_args(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("-data-dir", type=str, default='',
                        help="HDF5 prefix (<dir>_train.hdf5); synthetic data when absent")
    parser.add_argument("-epochs", type=int, default=1)
    parser.add_argument("-test-freq", type=int, default=1)
    parser.add_argument("-exp-name", type=str, default='piano_test')
    parser.add_argument("--n-train-read", type=int, default=None)
    parser.add_argument("--n-test-read", type=int, default=None)
    parser.add_argument("--batch-size", type=int, default=16)
    parser.add_argument("--frames", type=int, default=252)
    parser.add_argument("-loss", type=str, default="l1", choices=LOSSES,
                        help="l1 (train.py:132), the README's multi-scale spectral loss, or both")
    parser.add_argument("-mss-phase", type=str, default="griffinlim", choices=("griffinlim", "target"),
                        help="phase that renders the prediction for the multi-scale loss")
    parser.add_argument("-gl-iters", type=int, default=8,
                        help="Griffin-Lim iterations behind the multi-scale loss's audio")
    return parser.parse_args(argv)


if __name__ == "__main__":
    main(parse_args())


__all__ = ["train", "test", "Adam", "make_optimizer", "make_loss", "LOSSES", "hyperparams", "main",
           "np"]
