"""PerformanceNet / blocks / train step on the HIP path vs the golden fixtures made from the
reference model (tests/golden/make_golden.py imports /root/reference/model/model.py and runs it
in fp32 AND fp64).

This network's gradients are ill-conditioned in fp32: L1's sign(y-t), the LeakyReLU/ReLU kinks
and maxpool argmax ties flip whenever a value sits within rounding of the kink, so the
reference's OWN fp32 gradients differ from its fp64 ones by 1-16% (L2, per parameter). Parity
is therefore judged against the fp64 truth with the reference fp32 gap as the yardstick:
  loss                |ours - ref32| <= 1e-4 * |ref|          (north_star 1e-4 on loss values)
  outputs (sampled)   max|ours - ref64| <= max(4 * max|ref32 - ref64|, 1e-5 * max|ref64|)
  weight gradients    ||ours - g64|| / ||g64|| <= max(4 * ref32 gap, 1e-4)  on 256 samples/param;
                      IN-preceded conv biases (exact gradient 0) only bounded
  Adam after 1-2 steps |ours - ref| <= 2e-5 where |g64| is well above the fp32 noise floor
"""
import os

import numpy as np
import pytest
import torch

from oracle import detinit

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _noise_bias(name):
    """Conv biases followed by InstanceNorm: exact gradient 0 (IN removes the mean)."""
    return name.endswith(".bias") and not (name.startswith("dense_concats") or name == "lastconv.bias")


def _det_model(cuda):
    from ml_music_style_transfer_amd.model import PerformanceNet
    torch.manual_seed(0)
    net = PerformanceNet()
    sd = {n: torch.from_numpy(detinit.param_value(n, tuple(p.shape))) for n, p in net.named_parameters()}
    net.load_state_dict(sd)
    return net.to(cuda)


def _inputs(B, T, cuda):
    return [torch.from_numpy(a).to(cuda) for a in detinit.model_inputs(B, T)]


@pytest.mark.parametrize("fname", ["full_B2_T44.npz", "full_B1_T252.npz"])
def test_full_model_vs_golden(cuda, fname):
    from ml_music_style_transfer_amd import engine as E
    g = np.load(os.path.join(GOLD, fname))
    B, T = int(g["B"]), int(g["T"])
    net = _det_model(cuda)
    net.eval()
    assert [n for n, _ in net.named_parameters()] == list(g["param_names"])
    xm, xa, cd, tg = _inputs(B, T, cuda)
    y = net(xm, xa, cd)
    loss = E.l1_loss(y, tg)
    loss.backward()
    assert tuple(y.shape) == tuple(g["out_shape"])
    lv, lr = loss.item(), float(g["loss"])
    assert abs(lv - lr) <= 1e-4 * abs(lr), (lv, lr)
    yv = y.detach().double().cpu().numpy().ravel()[g["out_idx"]]
    y64, y32 = g["out_val64"], g["out_val"].astype(np.float64)
    lim = max(4 * np.abs(y32 - y64).max(), 1e-5 * np.abs(y64).max())
    assert np.abs(yv - y64).max() <= lim, (np.abs(yv - y64).max(), lim)
    report = []
    for n, p in net.named_parameters():
        if f"gnone:{n}" in g.files:
            assert p.grad is None, n
            continue
        assert p.grad is not None, n
        gv = p.grad.detach().double().cpu().numpy().ravel()[g[f"gidx:{n}"]]
        g64, g32 = g[f"gval64:{n}"], g[f"gval:{n}"].astype(np.float64)
        if _noise_bias(n):
            wscale = np.abs(g[f"gval64:{n.replace('.bias', '.weight')}"]).max()
            assert np.abs(gv).max() <= 1e-2 * wscale + 1e-9, n
            continue
        den = np.linalg.norm(g64) + 1e-30
        ours, theirs = np.linalg.norm(gv - g64) / den, np.linalg.norm(g32 - g64) / den
        report.append((ours, theirs, n))
        assert ours <= max(4 * theirs, 1e-4), (n, ours, theirs)
    report.sort()
    print("worst (ours, ref32) gap vs fp64:", report[-3:])


def test_adam_steps_vs_golden(cuda):
    from ml_music_style_transfer_amd import engine as E
    from ml_music_style_transfer_amd.train import make_optimizer
    g = np.load(os.path.join(GOLD, "full_B2_T44.npz"))
    net = _det_model(cuda)
    net.eval()
    opt = make_optimizer(net, lr=1e-3)
    xm, xa, cd, tg = _inputs(2, 44, cuda)
    checked = 0
    for step, key in ((1, "adam"), (2, "adam2")):
        opt.zero_grad()
        loss = E.l1_loss(net(xm, xa, cd), tg)
        loss.backward()
        opt.step()
        if step == 2:
            # Adam's first step is sign descent: every gradient element below the fp32 noise
            # floor moves +-lr at random, so the loss after it carries that noise. ref32 vs
            # ref64 is 1.2e-4 relative; two GPU summation orders of the same GEMMs (channel-
            # major and tap-major K) gave +1.4e-3 and -1.5e-3. Bound: 3e-3 relative to fp64.
            l32, l64 = float(g["loss2"]), float(g["loss2_64"])
            assert abs(loss.item() - l64) <= max(4 * abs(l32 - l64), 3e-3 * l64), (loss.item(), l32, l64)
        for n, p in net.named_parameters():
            if f"{key}:{n}" not in g.files or _noise_bias(n):
                continue
            g64 = np.abs(g[f"gval64:{n}"])
            gap = g[f"gstat:{n}"][3] / max(g[f"gstat:{n}"][4], 1e-30)  # ref32 L2 gap
            ok = g64 > max(20 * gap, 0.05) * g64.max()  # elements well above the fp32 noise
            v = p.detach().cpu().numpy().ravel()[g[f"gidx:{n}"]]
            # step 1 is strict; step 2's gradient is taken at parameters that already carry
            # step 1's sign noise, so it is only bounded to 1/4 of the cumulative update (2 lr)
            tol = 2e-5 if step == 1 else 5e-4
            assert np.abs(v - g[f"{key}:{n}"])[ok].max(initial=0) <= tol, (key, n)
            checked += int(ok.sum())
    assert checked > 300
    assert len(opt._flat_groups) == 1  # the fused flat path ran


def test_blocks_vs_golden(cuda):
    from ml_music_style_transfer_amd import model as M
    g = np.load(os.path.join(GOLD, "blocks.npz"))

    def load(mod, seed):
        mod.load_state_dict({n: torch.from_numpy(detinit.param_value(n, tuple(p.shape), seed))
                             for n, p in mod.named_parameters()})
        return mod.to(cuda)

    def T(a, req=False):
        return torch.from_numpy(a).to(cuda).requires_grad_(req)

    def chk(got, ref, tol=2e-5):
        ref = np.asarray(ref)
        scale = max(np.abs(ref).max(), 1e-6)
        assert np.abs(got.detach().cpu().numpy() - ref).max() <= tol * scale * 10

    for pool in (True, False):
        k = f"downconv_pool{int(pool)}"
        m = load(M.DownConv(5, 7, block_id=0, pooling=pool), 3)
        x = T(g[k + ":x"], True)
        y, before = m(x)
        r1 = torch.from_numpy(detinit.uniform("dc_r1", tuple(y.shape))).to(cuda)
        r2 = torch.from_numpy(detinit.uniform("dc_r2", tuple(before.shape))).to(cuda)
        ((y * r1).sum() + (before * r2).sum()).backward()
        chk(y, g[k + ":y"])
        chk(before, g[k + ":before"])
        chk(x.grad, g[k + ":dx"])
        for n, p in m.named_parameters():
            if n.endswith("bias"):
                continue
            chk(p.grad, g[k + ":d:" + n])

    for (kk, cond) in ((6, 3), (4, 2), (3, 0), (2, 0)):
        for dskip in (-3, -2, -1, 0, 1, 2, 3):
            k = f"upconv_k{kk}_d{dskip}"
            m = load(M.UpConv(6, 4, 3, cond, block_id=5, upconv_kernel=kk), 5)
            dec, res = T(g[k + ":dec"], True), T(g[k + ":res"], True)
            c = T(g[k + ":cond"], True) if cond else None
            y = m(res, dec, c)
            r = torch.from_numpy(detinit.uniform(f"uc_r{kk}{dskip}", tuple(y.shape))).to(cuda)
            (y * r).sum().backward()
            chk(y, g[k + ":y"])
            chk(dec.grad, g[k + ":ddec"])
            chk(res.grad, g[k + ":dres"])
            if cond:
                chk(c.grad, g[k + ":dcond"])
            for n, p in m.named_parameters():
                if not n.endswith("bias"):
                    chk(p.grad, g[k + ":d:" + n])

    m = load(M.DenseConcat(8, 6, 5), 7)
    m.eval()
    mid, aud = T(g["dense:midi"], True), T(g["dense:audio"], True)
    y = m(mid, aud)
    r = torch.from_numpy(detinit.uniform("dn_r", tuple(y.shape))).to(cuda)
    (y * r).sum().backward()
    chk(y, g["dense:y"])
    chk(mid.grad, g["dense:dmidi"])
    chk(aud.grad, g["dense:daudio"])
    for n, p in m.named_parameters():
        chk(p.grad, g["dense:d:" + n])

    m = load(M.MBRBlock(16, 4), 9)
    y = m(T(g["mbr:x"]))
    np.testing.assert_array_equal(y.cpu().numpy(), g["mbr:y"])

    m = load(M.Onset_Offset_Encoder(depth=3, start_channels=4), 11)
    x = T(g["onset:x"], True)
    conds = m(x)
    assert len(conds) == int(g["onset:n"])
    (sum((c * torch.from_numpy(detinit.uniform(f"oe_r{i}", tuple(c.shape))).to(cuda)).sum()
         for i, c in enumerate(conds))).backward()
    for i, c in enumerate(conds):
        chk(c, g[f"onset:c{i}"])
    chk(x.grad, g["onset:dx"])

    up = torch.from_numpy(g["crop:up"]).to(cuda)
    for d in range(-3, 4):
        out = M.UpConv.crop_and_concat(up, torch.from_numpy(g[f"crop:d{d}:byp"]).to(cuda))
        np.testing.assert_array_equal(out.cpu().numpy(), g[f"crop:d{d}:out"])


def test_train_dropin_runs(cuda):
    """train.py's train()/test() API end to end on synthetic batches (dropout on)."""
    from ml_music_style_transfer_amd import train as TR
    from ml_music_style_transfer_amd.model import PerformanceNet
    net = PerformanceNet().to(cuda)
    opt = TR.make_optimizer(net)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, "min")
    ds = TR.SyntheticSpectrogramDataset(4, T=44, seed=3)
    dl = torch.utils.data.DataLoader(ds, batch_size=2, shuffle=True)
    hist = []
    l0 = TR.train(net, 0, dl, opt, hist)
    l1 = TR.train(net, 1, dl, opt, hist)
    assert np.isfinite(hist).all() and len(hist) == 4
    assert l1.item() < l0.item()
    tl = TR.test(net, 0, dl, sched, [])
    assert np.isfinite(tl.item())


def test_adam_inside_backward_matches_step(cuda):
    """BackwardAdam (bucket updates on a side stream during backward) gives bitwise the same
    parameters, moments and losses as the one-launch update in step(), over three steps with
    small buckets (many launches, buckets ending inside the network)."""
    from ml_music_style_transfer_amd import engine as E
    from ml_music_style_transfer_amd.train import make_optimizer
    xm, xa, cd, tg = _inputs(2, 44, cuda)
    runs = []
    for overlap in (False, True):
        net = _det_model(cuda).eval()
        opt = make_optimizer(net, lr=1e-3)
        if overlap:
            opt.overlap_backward(bucket_bytes=8 << 20)
        losses = []
        for _ in range(3):
            opt.zero_grad()
            loss = E.l1_loss(net(xm, xa, cd), tg)
            loss.backward()
            opt.step()
            losses.append(loss.item())
        if overlap:
            assert opt._bwd.updates == 3 and len(opt._bwd.buckets) > 20
        pf, _, _ = net.flat_buffers()
        st = next(iter(opt._flat_groups.values()))
        runs.append((losses, pf.clone(), st["m"].clone(), st["v"].clone(), st["step"]))
    (l0, p0, m0, v0, s0), (l1, p1, m1, v1, s1) = runs
    assert l0 == l1 and s0 == s1 == 3
    assert torch.equal(p0, p1) and torch.equal(m0, m1) and torch.equal(v0, v1)


def test_wgrad_side_stream_bitwise(cuda):
    """Every concurrent stream layout of the training step produces bitwise the serial order's
    gradients and parameters, at the training batch's time axis, over three steps per network
    (from the second backward on, the weight-gradient tail of MST_WGRAD_MAIN_TAIL blocks runs on
    the home stream, since GradSink takes the block count from the previous backward):
    weight-gradient side stream on / off x encoder stream on / off, each without and with backward
    Adam on small (8 MB) buckets. Backward Adam with the side stream off and the encoder stream
    on is the layout where a bucket spanning a skip-level DenseConcat (written on the encoder
    stream) and the next up-convolution block (main stream) must wait for both writers
    (engine.GradSink.block_done)."""
    from ml_music_style_transfer_amd import engine as E
    from ml_music_style_transfer_amd import model as M
    from ml_music_style_transfer_amd.train import make_optimizer
    xm, xa, cd, tg = _inputs(2, 252, cuda)
    keep = (M._WGRAD_STREAM, M._ENC_STREAM)
    steps = 3

    def run(side, enc, overlap):
        M.set_wgrad_stream(side)
        M.set_enc_stream(enc)
        net = _det_model(cuda).eval()
        opt = make_optimizer(net, lr=1e-3)
        if overlap:
            opt.overlap_backward(bucket_bytes=8 << 20)
        for _ in range(steps):
            opt.zero_grad()
            E.l1_loss(net(xm, xa, cd), tg).backward()
            g = net.flat_buffers()[1].clone()
            opt.step()
            yield g, net.flat_buffers()[0].clone()

    try:
        for overlap in (False, True):
            ref = list(run(False, False, overlap))  # serial: one stream
            for side, enc in ((True, False), (False, True), (True, True)):
                for it, (g, p) in enumerate(run(side, enc, overlap)):
                    assert torch.equal(ref[it][0], g), (overlap, side, enc, it, "grad")
                    assert torch.equal(ref[it][1], p), (overlap, side, enc, it, "param")
                    del g, p
            del ref
            torch.cuda.empty_cache()
    finally:
        M.set_wgrad_stream(keep[0])
        M.set_enc_stream(keep[1])


def test_side_streams_joined_once_main_stream_synced(cuda):
    """Stream-ordering invariant of the default training step: every launch on the weight-gradient
    side stream (engine.GradSink) and on backward Adam's stream (train.BackwardAdam) is joined into
    the compute stream before backward / step() return, so synchronising the compute stream ALONE
    must complete the join events (each recorded on its side stream behind the last launch there):
    no side-stream kernel can still run (or fault) after the caller's last sync point. Checked after
    backward and after step(), with and without backward Adam, at the training batch's time axis.
    (The side stream itself may still hold the caching allocator's event markers for tensors
    recorded on it and freed after the join - events, not kernels - so Stream.query() is not the
    test: round 4's first version asserted it and saw a marker in flight.)"""
    from ml_music_style_transfer_amd import engine as E
    from ml_music_style_transfer_amd import model as M
    from ml_music_style_transfer_amd.train import make_optimizer
    xm, xa, cd, tg = _inputs(2, 252, cuda)
    keep = M._WGRAD_STREAM
    try:
        M.set_wgrad_stream(True)
        for overlap in (False, True):
            net = _det_model(cuda).train()
            opt = make_optimizer(net, lr=1e-3)
            if overlap:
                opt.overlap_backward(bucket_bytes=8 << 20)
            for _ in range(2):
                opt.zero_grad()
                E.l1_loss(net(xm, xa, cd), tg).backward()
                joined = net.__dict__["_mst_wgrad_joined"]
                assert joined is not None  # the side stream ran and was joined
                torch.cuda.current_stream().synchronize()
                assert joined.query(), "a weight-gradient launch outlived the compute-stream sync"
                opt.step()
                torch.cuda.current_stream().synchronize()
                if overlap:
                    assert opt._bwd.joined.query(), "a backward-Adam launch outlived step()'s sync"
            if overlap:
                assert opt._bwd.updates == 2
    finally:
        M.set_wgrad_stream(keep)


def test_backward_gradient_order_matches_flat_layout(cuda):
    """The flat gradient buffer is laid out in engine.backward_param_order so that
    data-parallel buckets complete front to back; check the backward program really
    produces gradients in that order, block by block, and the layout is ascending in it."""
    from ml_music_style_transfer_amd import engine as E
    net = _det_model(cuda).train()
    names = {id(p): n for n, p in net.named_parameters()}
    seen = []

    class Rec:
        def begin(self):
            pass

        def ready(self, params):
            seen.extend(names[id(p)] for p in params)

        def launch_remaining(self):
            pass

    net._mst_dp = Rec()
    xm, xa, cd, tg = _inputs(1, 44, cuda)
    y = net(xm, xa, cd)
    E.l1_loss(y, tg).backward()
    del net._mst_dp
    order = E.backward_param_order(net.depth)
    assert seen == order
    offs = [net._flat["index"][id(dict(net.named_parameters())[n])][0] for n in order]
    assert offs == sorted(offs)


def test_full_model_bench_config_B32(cuda):
    """The benchmarked configuration (bench.py: B=32, T=252) against the reference: fixture
    full_B32_T252.npz (make_golden.py bench: /root/reference/model/model.py run in fp32 and fp64
    on 32 distinct detinit samples, eval mode). At N = B*T = 8064 columns the GEMMs take the
    split-K and tile schedules the bench runs (checked below), none of which occur at B <= 2.
    Tolerances: loss 1e-4 relative; sampled outputs within the north_star's 1e-4 of the output
    scale (max abs) and 1e-4 relative L2 vs fp64 (the MFMA accumulator sums each K slab
    sequentially, so output error grows with the unsplit K length: tools/parity_probe.py
    measured rel L2 2.6e-5 at B=1 and 9.2e-5 with no split at all, vs the CPU reference's
    blocked fp32 sums at 1.9e-5; every single GEMM at these shapes is within 1.5e-6 of fp64,
    tests/test_gpu_bench_shapes.py); weight gradients within 4x the reference fp32 gap, as
    test_full_model_vs_golden."""
    from ml_music_style_transfer_amd import engine as E
    from ml_music_style_transfer_amd import kernels as K
    g = np.load(os.path.join(GOLD, "full_B32_T252.npz"))
    B, T = int(g["B"]), int(g["T"])
    assert (B, T) == (32, 252)
    net = _det_model(cuda).eval()
    xm, xa, cd, tg = _inputs(B, T, cuda)
    log = []
    K.gemm_timing(log)
    try:
        y = net(xm, xa, cd)
        loss = E.l1_loss(y, tg)
        loss.backward()
    finally:
        K.gemm_timing(None)
    torch.cuda.synchronize()
    split = [shp for *_, shp in log if shp and shp[-1] > 0]  # launches with a split-K workspace
    assert len(split) >= 5, "the B=32 schedules should split K on several layers"
    lv, lr = loss.item(), float(g["loss"])
    assert abs(lv - lr) <= 1e-4 * abs(lr), (lv, lr)
    y64, y32 = g["out_val64"], g["out_val"].astype(np.float64)
    yv = y.detach().double().cpu().numpy().ravel()[g["out_idx"]]
    err = np.abs(yv - y64).max()
    rel = np.linalg.norm(yv - y64) / np.linalg.norm(y64)
    print(f"B=32 outputs vs fp64: max {err:.3e} (ref fp32 {np.abs(y32 - y64).max():.3e}); rel L2 "
          f"{rel:.3e} (ref fp32 {np.linalg.norm(y32 - y64) / np.linalg.norm(y64):.3e})")
    assert err <= 1e-4 * np.abs(y64).max(), (err, np.abs(y64).max())
    assert rel <= 1e-4, rel
    worst = []
    for n, p in net.named_parameters():
        if f"gnone:{n}" in g.files:
            assert p.grad is None, n
            continue
        gv = p.grad.detach().double().cpu().numpy().ravel()[g[f"gidx:{n}"]]
        g64, g32 = g[f"gval64:{n}"], g[f"gval:{n}"].astype(np.float64)
        if _noise_bias(n):
            wscale = np.abs(g[f"gval64:{n.replace('.bias', '.weight')}"]).max()
            assert np.abs(gv).max() <= 1e-2 * wscale + 1e-9, n
            continue
        den = np.linalg.norm(g64) + 1e-30
        ours, theirs = np.linalg.norm(gv - g64) / den, np.linalg.norm(g32 - g64) / den
        worst.append((ours / max(theirs, 2.5e-5), ours, theirs, n))
    worst.sort()
    print("B=32: split-K launches", len(split), "worst (ratio, ours, ref32) vs fp64:", worst[-4:])
    for ratio, ours, theirs, n in worst:
        assert ours <= max(4 * theirs, 1e-4), (n, ours, theirs)


def _full_vs_fp64(net, g, y, loss):
    """Loss, sampled outputs and sampled weight gradients vs a make_golden.py full_model_lowmem
    fixture, with test_full_model_bench_config_B32's bounds. Returns the worst gradient rows."""
    lv, lr = loss.item(), float(g["loss"])
    assert abs(lv - lr) <= 1e-4 * abs(lr), (lv, lr)
    assert tuple(y.shape) == tuple(g["out_shape"])
    y64, y32 = g["out_val64"], g["out_val"].astype(np.float64)
    yv = y.detach().double().cpu().numpy().ravel()[g["out_idx"]]
    err = np.abs(yv - y64).max()
    rel = np.linalg.norm(yv - y64) / np.linalg.norm(y64)
    assert err <= 1e-4 * np.abs(y64).max(), (err, np.abs(y64).max())
    assert rel <= 1e-4, rel
    worst = []
    for n, p in net.named_parameters():
        if f"gnone:{n}" in g.files:
            assert p.grad is None, n
            continue
        gv = p.grad.detach().double().cpu().numpy().ravel()[g[f"gidx:{n}"]]
        g64, g32 = g[f"gval64:{n}"], g[f"gval:{n}"].astype(np.float64)
        if _noise_bias(n):
            wscale = np.abs(g[f"gval64:{n.replace('.bias', '.weight')}"]).max()
            assert np.abs(gv).max() <= 1e-2 * wscale + 1e-9, n
            continue
        den = np.linalg.norm(g64) + 1e-30
        ours, theirs = np.linalg.norm(gv - g64) / den, np.linalg.norm(g32 - g64) / den
        worst.append((ours / max(theirs, 2.5e-5), ours, theirs, n))
        assert ours <= max(4 * theirs, 1e-4), (n, ours, theirs)
    worst.sort()
    return err, rel, worst[-3:]


@pytest.mark.parametrize("fname", ["full_B2_T860.npz", "full_B2_T100.npz"])
def test_full_model_reference_lengths(cuda, fname):
    """The reference's own training length and an off-grid one, vs the reference model
    (make_golden.py t860: /root/reference/model/model.py in fp32 and fp64), bounds as in
    test_full_model_bench_config_B32.
    T = 860: 5 s @ 44.1 kHz = spc * wps frames (preprocess.py:24-25,40-42,66,86), the chunk the
    reference trains on; its levels run at T = 860/430/215/107/53, so the deep layers take
    split-K schedules and odd-length InstanceNorm rows the T = 44/252 fixtures never reach.
    T = 100: 100 = 4 (mod 16), so the U-Net returns 16 * 6 + 12 = 108 frames (model.py:229-232),
    the case the inference CLI meets on whole tracks; the L1 target is drawn at 108 frames."""
    from ml_music_style_transfer_amd import engine as E
    from ml_music_style_transfer_amd import kernels as K
    g = np.load(os.path.join(GOLD, fname))
    B, T = int(g["B"]), int(g["T"])
    net = _det_model(cuda).eval()
    xm, xa, cd, tg = _inputs(B, T, cuda)
    Tout = int(g["out_shape"][2])
    if Tout != T:
        tg = torch.from_numpy(detinit.offgrid_target(B, Tout)).to(cuda)
    log = []
    K.gemm_timing(log)
    try:
        y = net(xm, xa, cd)
        loss = E.l1_loss(y, tg)
        loss.backward()
    finally:
        K.gemm_timing(None)
    torch.cuda.synchronize()
    err, rel, worst = _full_vs_fp64(net, g, y, loss)
    split = sorted({(tag, *shp[:3], round(shp[-1] / (4.0 * shp[0] * shp[1]), 2))
                    for _, _, _, tag, shp in log if shp and shp[-1] > 0})
    print(f"B={B} T={T}: out {tuple(y.shape)}, max {err:.3e}, rel L2 {rel:.3e}; "
          f"{len(log)} GEMM launches, split-K schedules (kind, M, N, K, splits): {split}; worst {worst}")


def test_train_steps_reference_batch_B16_T860(cuda):
    """The reference's default training shape: --batch-size 16 (train.py:219) on 860-frame
    chunks (preprocess.py:42,66).
    Against the reference itself (round 6): full_B16_T860.npz (make_golden.py b16t860:
    /root/reference/model/model.py in fp32 and fp64 on these 16 detinit samples, eval mode) with
    test_full_model_bench_config_B32's bounds: loss 1e-4 relative, sampled outputs within 1e-4 of
    the output scale and 1e-4 relative L2 vs fp64, sampled weight gradients within 4x the
    reference's own fp32-vs-fp64 gap per parameter.
    Properties on top: samples are independent (InstanceNorm is per sample, train.py:132's L1 is
    a mean), so the B = 16 loss equals the mean of its two B = 8 halves' losses (1e-5 relative)
    and its weight gradients the mean of theirs. The halves run other split-K schedules, i.e.
    other fp32 summation orders, and this network's fp32 gradients are ill-conditioned (L1 sign,
    ReLU / LeakyReLU kinks, maxpool ties flip under rounding), so each parameter's rel L2 gap is
    held to 4x the reference's own fp32-vs-fp64 gap for that parameter at T = 860 (full_B2_T860
    .npz), floor 1e-3. Then three Adam steps on the batch stay finite and lower the loss."""
    from ml_music_style_transfer_amd import engine as E
    from ml_music_style_transfer_amd.train import make_optimizer
    B, T = 16, 860
    xm, xa, cd, tg = _inputs(B, T, cuda)
    net = _det_model(cuda).eval()
    grads, losses = [], []
    for sl in (slice(0, B), slice(0, B // 2), slice(B // 2, B)):
        net.zero_grad(set_to_none=True)
        y = net(xm[sl], xa[sl], cd[sl])
        loss = E.l1_loss(y, tg[sl])
        loss.backward()
        if sl.start == 0 and sl.stop == B:
            err, rel, worst_ref = _full_vs_fp64(net, np.load(os.path.join(GOLD, "full_B16_T860.npz")),
                                                y, loss)
            print(f"B=16 T=860 vs the reference: out max {err:.3e}, rel L2 {rel:.3e}; worst "
                  f"(ratio to ref fp32 gap, ours, ref fp32 gap, name) {worst_ref}")
        del y
        losses.append(loss.item())
        grads.append({n: p.grad.detach().double().clone() for n, p in net.named_parameters()
                      if p.grad is not None})
    assert abs(losses[0] - 0.5 * (losses[1] + losses[2])) <= 1e-5 * abs(losses[0]), losses
    fx = np.load(os.path.join(GOLD, "full_B2_T860.npz"))
    worst = []
    for n, g0 in grads[0].items():
        if _noise_bias(n):
            continue
        gh = 0.5 * (grads[1][n] + grads[2][n])
        r = ((g0 - gh).norm() / (gh.norm() + 1e-30)).item()
        gap = float(fx[f"gstat:{n}"][3] / max(fx[f"gstat:{n}"][4], 1e-30))  # ref fp32 vs fp64
        worst.append((r / max(gap, 2.5e-4), r, gap, n))
        assert r <= max(4 * gap, 1e-3), (n, r, gap)
    worst = sorted(worst)[-3:]
    opt = make_optimizer(net, lr=1e-3)
    hist = []
    for _ in range(3):
        opt.zero_grad()
        loss = E.l1_loss(net(xm, xa, cd), tg)
        loss.backward()
        opt.step()
        hist.append(loss.item())
    assert all(np.isfinite(hist)) and hist[-1] < hist[0], hist
    assert all(torch.isfinite(p).all() for p in net.parameters())
    print(f"B=16 T=860: loss {losses[0]:.6f} = mean of halves {losses[1]:.6f}, {losses[2]:.6f}; "
          f"worst (ratio to ref fp32 gap, rel L2 vs halves, gap, name) {worst}; Adam losses {hist}")


def _grads_once(cuda):
    """A deterministic PerformanceNet and one backward's gradients (B=1, T=44, eval)."""
    from ml_music_style_transfer_amd import engine as E
    net = _det_model(cuda).eval()
    xm, xa, cd, tg = _inputs(1, 44, cuda)
    E.l1_loss(net(xm, xa, cd), tg).backward()
    return net


def test_adam_two_param_groups_matches_torch(cuda):
    """train.Adam's per-parameter path (taken with two param groups) on the real model, whose 3-D
    conv weights are tap-major slot views: after 3 steps on fixed gradients it equals the fused
    flat-buffer path bitwise and torch.optim.Adam (foreach=False) to fp32 rounding (measured 3
    ulps after 3 steps: the kernel's fused multiply-adds round each update differently; bound
    1e-6 relative + 1e-7, i.e. 1e-4 of one lr=1e-3 step) on every parameter, tap-major or not
    (train.py:188). A layout mix-up moves elements by the full 1e-3 step."""
    from ml_music_style_transfer_amd.train import Adam, make_optimizer
    results = []
    for mode in ("groups", "flat", "torch"):
        net = _grads_once(cuda)
        named = [(n, p) for n, p in net.named_parameters() if p.grad is not None]
        if mode == "groups":
            g1 = [p for n, p in named if n.startswith("down_convs_audio")]
            g2 = [p for n, p in named if not n.startswith("down_convs_audio")]
            opt = Adam([{"params": g1}, {"params": g2}], lr=1e-3).attach(net)
        elif mode == "flat":
            opt = make_optimizer(net, lr=1e-3)
        else:
            opt = torch.optim.Adam([p for _, p in named], lr=1e-3, foreach=False)
        for _ in range(3):
            opt.step()
        if mode == "groups":
            assert len(opt._flat_groups) == 0  # the per-parameter path ran
            assert any(not p.is_contiguous() for _, p in named)  # tap-major slots among them
        elif mode == "flat":
            assert len(opt._flat_groups) == 1
        torch.cuda.synchronize()
        results.append({n: p.detach().clone() for n, p in named})
        del net, opt
    ours, flat, ref = results
    for n in ref:
        assert torch.equal(ours[n], flat[n]), n
        torch.testing.assert_close(ours[n], ref[n], rtol=1e-6, atol=1e-7, msg=n)


def test_adam_flat_then_per_parameter_step_counts(cuda):
    """A fused flat step followed by a per-parameter step (taken when one parameter has no
    gradient) counts steps per parameter like torch.optim.Adam: the flat path gives each
    parameter its own step tensor, so the per-parameter `step += 1` moves only its own count."""
    from ml_music_style_transfer_amd.train import make_optimizer
    results = []
    for mode in ("ours", "torch"):
        net = _grads_once(cuda)
        named = [(n, p) for n, p in net.named_parameters() if p.grad is not None]
        if mode == "ours":
            opt = make_optimizer(net, lr=1e-3)
        else:
            opt = torch.optim.Adam([p for _, p in named], lr=1e-3, foreach=False)
        opt.step()                       # every parameter has a gradient: the flat path
        if mode == "ours":
            assert len(opt._flat_groups) == 1
        net.lastconv.bias.grad = None    # per-parameter path for the second step
        opt.step()
        torch.cuda.synchronize()
        results.append(({n: float(opt.state[p]["step"]) for n, p in named},
                        {n: p.detach().clone() for n, p in named}))
        del net, opt
    (s_ours, p_ours), (s_ref, p_ref) = results
    assert s_ours == s_ref
    assert s_ref["lastconv.bias"] == 1.0 and s_ref["lastconv.weight"] == 2.0
    for n in p_ref:
        torch.testing.assert_close(p_ours[n], p_ref[n], rtol=1e-6, atol=1e-7, msg=n)


def test_adam_state_dict_resume(cuda, tmp_path):
    """Optimizer checkpoint round trip (train.py:202-208 saves optimizer.state_dict()): two steps,
    save, a fresh model + optimizer loads both state_dicts, a third step; equals three
    uninterrupted steps bitwise (moments and bias-correction step count survive the fused
    flat-buffer state)."""
    from ml_music_style_transfer_amd import engine as E
    from ml_music_style_transfer_amd.train import make_optimizer
    xm, xa, cd, tg = _inputs(1, 44, cuda)

    def step(net, opt):
        opt.zero_grad()
        E.l1_loss(net(xm, xa, cd), tg).backward()
        opt.step()

    net = _det_model(cuda).eval()
    opt = make_optimizer(net)
    for _ in range(3):
        step(net, opt)
    ref = net.flat_buffers()[0].clone()

    net = _det_model(cuda).eval()
    opt = make_optimizer(net)
    for _ in range(2):
        step(net, opt)
    ck = tmp_path / "checkpoint-2.tar"
    torch.save({"state_dict": net.state_dict(), "optimizer": opt.state_dict()}, ck)
    del net, opt
    state = torch.load(ck, weights_only=True)
    net2 = _det_model(cuda).eval()
    net2.load_state_dict(state["state_dict"])
    opt2 = make_optimizer(net2)
    opt2.load_state_dict(state["optimizer"])
    step(net2, opt2)
    assert next(iter(opt2._flat_groups.values()))["step"] == 3
    assert torch.equal(net2.flat_buffers()[0], ref)


def test_adam_prepare_is_bitwise_neutral(cuda):
    """Adam.prepare() allocates the flat moments before the first step; two steps after it
    match two steps of an optimizer that allocates them lazily, bitwise."""
    from ml_music_style_transfer_amd.train import make_optimizer
    out = []
    for prep in (False, True):
        net = _grads_once(cuda)
        opt = make_optimizer(net, lr=1e-3)
        if prep:
            opt.prepare()
            assert len(opt._flat_groups) == 1
        opt.step()
        opt.step()
        torch.cuda.synchronize()
        out.append(net.flat_buffers()[0].clone())
        del net, opt
    assert torch.equal(out[0], out[1])
