"""Overlapped data-parallel gradient all-reduce on the real backward program, two ranks on one
GPU. RCCL needs one GPU per rank, so the collectives here run over gloo (device tensors, SUM
then scale); bench.py's N > 1 runs use the same OverlappedAllReduce over RCCL ("nccl", AVG).
Checks that the averaged gradients equal the mean of each rank's local gradients.
"""
import os
import queue
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

NSAMP = 200_000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import faulthandler
    import sys
    faulthandler.dump_traceback_later(240, exit=True, file=sys.stderr)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ml_music_style_transfer_amd import _lib, dp
    from ml_music_style_transfer_amd import engine as E
    from ml_music_style_transfer_amd.model import PerformanceNet
    from oracle import detinit
    _lib.load()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = PerformanceNet().to(dev).eval()   # eval: no dropout, so the two passes agree
    dp.broadcast_parameters(net)
    _, grad, n = net.flat_buffers()
    idx = torch.randint(0, n, (NSAMP,), generator=torch.Generator().manual_seed(3)).to(dev)
    xm, xa, cd, tg = [torch.from_numpy(a).to(dev) for a in detinit.model_inputs(1, 44)]
    xa = xa * (1.0 + 0.5 * rank)           # different data per rank

    def fwd_bwd():
        net.zero_grad(set_to_none=True)
        y = net(xm, xa, cd)
        E.l1_loss(y, tg).backward()

    fwd_bwd()
    local = grad[idx].cpu()
    r = dp.enable_overlapped_allreduce(net, bucket_bytes=64 << 20)
    fwd_bwd()
    issued_in_backward = r.next
    dp.finish_gradients(net)
    torch.cuda.synchronize()
    # numpy: pickled by value (a CPU tensor travels as a shared-memory fd that the parent can only
    # open while this process is alive)
    q.put((rank, local.numpy(), grad[idx].cpu().numpy(), issued_in_backward, len(r.buckets)))
    dist.barrier()
    dist.destroy_process_group()


def test_overlapped_allreduce_two_ranks_one_gpu(cuda):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    deadline = time.monotonic() + 300
    while len(res) < world:
        try:
            rank, local, reduced, issued, nb = q.get(timeout=5)
            res[rank] = (torch.from_numpy(local), torch.from_numpy(reduced), issued, nb)
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead or time.monotonic() > deadline:
                for p in procs:
                    p.kill()
                pytest.fail(f"worker failed (exit codes {dead})")
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    mean = (res[0][0] + res[1][0]) / 2
    assert not torch.equal(res[0][0], res[1][0])
    for r in range(world):
        local, reduced, issued, nb = res[r]
        assert nb > 10 and issued == nb  # every bucket was issued by the end of backward
        torch.testing.assert_close(reduced, mean, rtol=1e-5, atol=1e-9)


def _train_worker(rank, world, port, workdir, q):
    import faulthandler
    import sys
    faulthandler.dump_traceback_later(280, exit=True, file=sys.stderr)
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "MST_DIST_BACKEND": "gloo"})
    os.chdir(workdir)
    from ml_music_style_transfer_amd import train as TR
    hp, model = TR.main(TR.parse_args(["-data-dir", os.path.join(workdir, "piano"), "-epochs",
                                       "2", "--batch-size", "2"]), return_model=True)
    flat, _, n = model.flat_buffers()
    idx = torch.randint(0, n, (NSAMP,), generator=torch.Generator().manual_seed(4)).to(flat.device)
    torch.cuda.synchronize()
    q.put((rank, hp.loss_history, hp.test_loss_history, hp.best_epoch,
           flat[idx].cpu().numpy()))  # numpy: pickled by value, no fd sharing
    dist.barrier()
    dist.destroy_process_group()


def test_train_main_data_parallel_two_ranks(cuda, tmp_path, monkeypatch):
    """train.main under WORLD_SIZE=2 (train.py:173-208 + SURVEY §8(e)): rank 0's weights
    broadcast, DistributedSampler shards of the HBM-resident HDF5 split, overlapped gradient
    all-reduce, loss sums over ranks, checkpoint from rank 0 only. After two epochs both
    ranks hold identical weights and report identical epoch losses."""
    import numpy as np
    from ml_music_style_transfer_amd import data, train as TR
    rng = np.random.default_rng(8)
    for split, N in (("train", 8), ("test", 4)):
        T = 44
        pr = (rng.random((N, T, 128)) < 0.1).astype(float)
        oo = np.diff(np.concatenate([np.zeros((N, 1, 128)), pr], 1), axis=1)
        data.write_split(str(tmp_path / ("piano_%s.hdf5" % split)), pr, oo,
                         {"cuba": 2 * rng.random((N, 1025, T)), "upright": 2 * rng.random((N, 1025, T))})
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_train_worker, args=(r, world, port, str(tmp_path), q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    deadline = time.monotonic() + 300
    while len(res) < world:
        try:
            r, lh, th, be, pr_ = q.get(timeout=5)
            res[r] = (lh, th, be, pr_)
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead or time.monotonic() > deadline:
                for p in procs:
                    p.kill()
                pytest.fail(f"worker failed (exit codes {dead})")
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res[0][0] == res[1][0] and res[0][1] == res[1][1] and res[0][2] == res[1][2]
    assert all(np.isfinite(res[0][0])) and len(res[0][0]) == 2
    np.testing.assert_array_equal(res[0][3], res[1][3])
    exp = tmp_path / "experiments" / "piano_test"
    assert (exp / ("checkpoint-%d.tar" % res[0][2])).exists() and (exp / "hyperparams.json").exists()


def _variants_worker(rank, world, port, q, emulate_rccl=False):
    """Three data-parallel update paths on the same two steps, and gradient accumulation.
    emulate_rccl: dp's RCCL-only branches (native AVG, BackwardAdam waiting on works[b] with no
    scale) over gloo through tests/_rccl_emulation.py."""
    import faulthandler
    import sys
    faulthandler.dump_traceback_later(280, exit=True, file=sys.stderr)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ml_music_style_transfer_amd import _lib, dp
    if emulate_rccl:
        import _rccl_emulation
        dp = _rccl_emulation.install()
    from ml_music_style_transfer_amd import engine as E
    from ml_music_style_transfer_amd.model import PerformanceNet
    from ml_music_style_transfer_amd.train import make_optimizer
    from oracle import detinit
    _lib.load()
    dev = torch.device("cuda", 0)
    xm, xa, cd, tg = [torch.from_numpy(a).to(dev) for a in detinit.model_inputs(1, 44)]
    xa = xa * (1.0 + 0.5 * rank)           # different data per rank

    def fresh():
        torch.manual_seed(0)
        net = PerformanceNet().to(dev).eval()   # eval: no dropout
        dp.broadcast_parameters(net)
        return net

    def loss_of(net, k=0):
        return E.l1_loss(net(xm, xa * (1.0 + 0.25 * k), cd), tg)

    finals = {}
    for mode in ("step", "backward_adam", "post"):
        net = fresh()
        if mode != "post":
            dp.enable_overlapped_allreduce(net, bucket_bytes=64 << 20)
        opt = make_optimizer(net, lr=1e-3, overlap_backward=(mode == "backward_adam"))
        for _ in range(2):
            opt.zero_grad()
            loss_of(net).backward()
            if mode == "post":
                dp.allreduce_gradients(net)
            opt.step()
        if mode == "backward_adam":
            assert opt._bwd.updates == 2  # the bucket updates ran inside backward, on gloo
        finals[mode] = net.flat_buffers()[0].clone()
        del net, opt
    same = [torch.equal(finals["step"], finals[m]) for m in ("backward_adam", "post")]
    n = finals["step"].numel()
    idx = torch.randint(0, n, (NSAMP,), generator=torch.Generator().manual_seed(5)).to(dev)
    sample = finals["step"][idx].cpu().numpy()  # numpy: pickled by value, no fd sharing
    del finals

    # gradient accumulation: two backward passes per step with the overlapped reducer equal the
    # post-backward average of the accumulated local gradients
    acc = {}
    for mode in ("overlapped", "post"):
        net = fresh()
        if mode == "overlapped":
            dp.enable_overlapped_allreduce(net, bucket_bytes=64 << 20)
        net.zero_grad(set_to_none=True)
        loss_of(net, 0).backward()
        loss_of(net, 1).backward()
        if mode == "post":
            dp.allreduce_gradients(net)
        else:
            dp.finish_gradients(net)
        acc[mode] = net.flat_buffers()[1][idx].cpu().numpy()
        del net
    torch.cuda.synchronize()
    q.put((rank, same, sample, acc["overlapped"], acc["post"]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("emulate_rccl", [False, True])
def test_dp_update_paths_bitwise_two_ranks_one_gpu(cuda, emulate_rccl):
    """Two ranks over gloo on one GPU exercise every data-parallel branch bench.py and train.main
    take over RCCL: the overlapped bucket reducer with Adam in step(), BackwardAdam (each bucket's
    update on a side stream right after that bucket's average, inside backward) and the
    post-backward all-reduce. After two steps all three hold bitwise the same parameters, on
    both ranks. With two backward passes before the exchange the overlapped reducer's result
    equals the average of the accumulated gradients (fp32 rounding: 1e-5 relative).
    With emulate_rccl the same holds on the branches only RCCL takes (ReduceOp.AVG issued,
    BackwardAdam's side stream waiting on works[b] with no scale of its own)."""
    import numpy as np
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_variants_worker, args=(r, world, port, q, emulate_rccl))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    deadline = time.monotonic() + 300
    while len(res) < world:
        try:
            rank, *rest = q.get(timeout=5)
            res[rank] = rest
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead or time.monotonic() > deadline:
                for p in procs:
                    p.kill()
                pytest.fail(f"worker failed (exit codes {dead})")
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in range(world):
        same, sample, acc_o, acc_p = res[r]
        assert same == [True, True], same
        np.testing.assert_allclose(acc_o, acc_p, rtol=1e-5, atol=1e-9)
    np.testing.assert_array_equal(res[0][1], res[1][1])


def test_bench_aux_two_ranks_one_gpu(tmp_path):
    """bench_aux.py under torch.distributed.run with 2 ranks (gloo rehearsal on one GPU): every
    rank takes its own clips, no data-path collective, one JSON line per workload from rank 0
    with n_gpus 2 and value = both ranks' clips over the max-over-ranks time. Unmeasured on
    xGMI hardware: this only proves the multi-rank harness runs."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MST_BENCH_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(root, "bench_aux.py"), "--workload", "frontend", "--clips", "16",
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 2
    for ln in lines:
        assert ln["n_gpus"] == 2 and ln["value"] > 0 and ln["config"]["clips_per_gpu"] == 16


@pytest.mark.timeout(300)
def test_bench_two_ranks_one_gpu(tmp_path):
    """bench.py exactly as the driver launches it for N > 1 (python -m torch.distributed.run
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 ... bench.py --gpus 2), rehearsed with
    MST_BENCH_BACKEND=gloo so both ranks can share this box's one GPU: rank 0 prints ONE JSON
    line with n_gpus 2, global batch 2 x 32, "dp2", value = both ranks' frames over the
    max-over-ranks step time, and an all-reduce object (bus bandwidth, exposed communication)
    without an error. The numbers are gloo-through-host numbers, NOT xGMI measurements: this only
    proves the multi-rank bench path runs (the step being sharded is reference
    model/train.py:129-143)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MST_BENCH_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--no-aux", "--no-cpu-baseline", "--kernel-timing-steps", "0"]
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    ln = lines[0]
    assert ln["n_gpus"] == 2 and ln["steps"] == 2 and ln["warmup"] == 1
    assert ln["config"]["global_batch"] == 64 and ln["config"]["parallelism"] == "dp2"
    assert ln["scaling"] == "weak" and ln["value"] > 0
    assert abs(ln["value"] - 64 * 252 / (ln["ms_per_step"] / 1000.0)) <= 1e-3 * ln["value"]
    ar = ln["allreduce"]
    assert "error" not in ar, ar
    assert ar["bus_GBps"] > 0 and "exposed_comm_ms_per_step" in ar and ar["overlapped"] is True
    # the flat gradient buffer: 726,039,425 live parameters in 16-byte aligned slots
    assert 4 * 726_039_425 <= ar["grad_bytes"] < 4 * 726_039_425 + 16 * 1000


def _ws4_worker(rank, world, port, q):
    """World size 4 with the bench's N > 1 update path: the overlapped bucket reducer plus Adam per
    bucket inside backward (train.BackwardAdam), over gloo on one GPU."""
    import faulthandler
    import sys
    faulthandler.dump_traceback_later(380, exit=True, file=sys.stderr)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ml_music_style_transfer_amd import _lib, dp
    from ml_music_style_transfer_amd import engine as E
    from ml_music_style_transfer_amd.model import PerformanceNet
    from ml_music_style_transfer_amd.train import make_optimizer
    from oracle import detinit
    from oracle import model_ref as R
    _lib.load()
    dev = torch.device("cuda", 0)
    xm, xa, cd, tg = [torch.from_numpy(a).to(dev) for a in detinit.model_inputs(1, 44)]

    def scale(r):  # different data per rank
        return 1.0 + 0.5 * r

    def make():
        torch.manual_seed(0)  # the same initial weights in every process
        return PerformanceNet().to(dev).eval()  # eval: no dropout

    def grads64(net):
        return {k: p.grad.detach().double().cpu() for k, p in net.named_parameters()
                if p.grad is not None}

    def rel_err(g, ref):
        num = sum(float((g[k] - ref[k]).square().sum()) for k in ref)
        den = sum(float(ref[k].square().sum()) for k in ref)
        return (num / den) ** 0.5

    n = make().flat_buffers()[2]
    idx = torch.randint(0, n, (NSAMP,), generator=torch.Generator().manual_seed(6)).to(dev)
    # this rank's local gradient, no exchange
    net = make()
    net.zero_grad(set_to_none=True)
    E.l1_loss(net(xm, xa * scale(rank), cd), tg).backward()
    local = net.flat_buffers()[1][idx].cpu().numpy()
    del net
    # rank 0: the gradient of the concatenated global batch (B = 4: the reference's step over the
    # whole batch, model/train.py:129-135; InstanceNorm is per sample and L1 a mean of equal-size
    # per-rank means, so it is the mean of the ranks' gradients), by ONE process in fp32 (this
    # library) and in float64 (oracle/model_ref.py on the CPU, the same weights)
    g4 = g64 = None
    if rank == 0:
        net = make()
        net.zero_grad(set_to_none=True)
        cat = lambda t: torch.cat([t] * world, 0)  # noqa: E731
        xa4 = torch.cat([xa * scale(r) for r in range(world)], 0)
        E.l1_loss(net(cat(xm), xa4, cat(cd)), cat(tg)).backward()
        g4 = grads64(net)
        p64 = {k: p.detach().double().cpu().requires_grad_(True) for k, p in net.named_parameters()}
        del net
        y64 = R.forward(p64, cat(xm).double().cpu(), xa4.double().cpu(), cat(cd).double().cpu())
        R.l1_loss(y64, cat(tg).double().cpu()).backward()
        g64 = {k: p64[k].grad for k in g4}
        del p64, y64
    # the data-parallel run: broadcast, overlapped reducer, backward Adam; two steps
    net = make()
    dp.broadcast_parameters(net)
    dp.enable_overlapped_allreduce(net, bucket_bytes=64 << 20)
    opt = make_optimizer(net, lr=1e-3, overlap_backward=True)
    reduced = errs = None
    for step in range(2):
        opt.zero_grad()
        E.l1_loss(net(xm, xa * scale(rank), cd), tg).backward()
        opt.step()
        if step == 0:
            reduced = net.flat_buffers()[1][idx].cpu().numpy()
            if rank == 0:
                errs = (rel_err(grads64(net), g64), rel_err(g4, g64))
    del g4, g64
    updates = opt._bwd.updates
    params = net.flat_buffers()[0][idx].cpu().numpy()
    torch.cuda.synchronize()
    q.put((rank, local, reduced, params, updates, errs))  # numpy: pickled by value
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(420)
def test_dp_four_ranks_global_batch_identity(cuda):
    """World size 4 (gloo, four ranks sharing one GPU) on the path bench.py and train.main take
    for N > 1: bucket all-reduces issued inside backward and each bucket's Adam update right after
    its average, inside backward. Checks, in eval mode:
      - every rank's averaged gradient equals the mean of the four local gradients (fp32
        rounding of the sum: 1e-5 relative, 200,000 sampled parameters);
      - it equals ONE process's gradient on the concatenated global batch of 4 within fp32
        tolerance. That tolerance is this network's own: its fp32 gradients are ill-conditioned
        (L1 signs, LeakyReLU kinks, maxpool ties; the conv biases ahead of each InstanceNorm have a
        true gradient of 0, so theirs is rounding noise), and two fp32 computations that sum in
        different orders (torch CPU, batch 4 vs four batches of 1) differ by 8.4 % in relative L2
        over all parameters. So both are measured against the float64 gradient of the global
        batch (oracle/model_ref.py, same weights): the averaged gradient's relative L2 error must be
        at most 2x that of the single-process fp32 batch-4 gradient ("Gradient
        conditioning", bounds the fixture tests the same way, per parameter at 4x);
      - both steps' updates ran inside backward, and after two steps all four ranks hold
        bit-identical parameters."""
    import numpy as np
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ws4_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    deadline = time.monotonic() + 400
    while len(res) < world:
        try:
            rank, *rest = q.get(timeout=5)
            res[rank] = rest
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead or time.monotonic() > deadline:
                for p in procs:
                    p.kill()
                pytest.fail(f"worker failed (exit codes {dead})")
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    mean = sum(res[r][0].astype(np.float64) for r in range(world)) / world
    assert not np.array_equal(res[0][0], res[1][0])
    for r in range(world):
        _, reduced, params, updates, _ = res[r]
        assert updates == 2, updates
        np.testing.assert_allclose(reduced, mean, rtol=1e-5, atol=1e-9)
        np.testing.assert_array_equal(params, res[0][2])
    e_dp, e_4 = res[0][4]
    print(f"relative L2 vs the float64 global-batch gradient: data-parallel average {e_dp:.3e}, "
          f"one process at batch {world} {e_4:.3e}")
    assert e_dp <= 2.0 * e_4, (e_dp, e_4)


@pytest.mark.timeout(420)
def test_bench_four_ranks_one_gpu(tmp_path):
    """bench.py as the driver launches it for N = 4 (torch.distributed.run --nproc-per-node 4 ...
    bench.py --gpus 4), rehearsed over gloo with the four ranks on this box's one GPU and a small
    per-rank batch (--batch 4): one JSON line from rank 0 with n_gpus 4, global batch 16, dp4, the
    value formula, and the all-reduce object. Gloo-through-host numbers, not xGMI ones."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MST_BENCH_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(root, "bench.py"), "--gpus", "4", "--batch", "4", "--steps", "2",
           "--warmup", "1", "--no-aux", "--no-cpu-baseline", "--kernel-timing-steps", "0"]
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    ln = lines[0]
    assert ln["n_gpus"] == 4 and ln["config"]["global_batch"] == 16
    assert ln["config"]["parallelism"] == "dp4" and ln["config"]["batch_per_gpu"] == 4
    assert abs(ln["value"] - 16 * 252 / (ln["ms_per_step"] / 1000.0)) <= 1e-3 * ln["value"]
    ar = ln["allreduce"]
    assert "error" not in ar, ar
    assert ar["bus_GBps"] > 0 and ar["overlapped"] is True
