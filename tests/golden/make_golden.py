"""Generate the golden parity fixtures from the REAL reference model.

Runs only in the build container, where /root/reference exists: it imports
/root/reference/model/model.py (PerformanceNet and its blocks; torch CPU) and
writes small .npz files next to this script. Only the fixtures (data) are
committed; no reference source or bytecode is copied. The GPU box never runs
this script.

Weights and inputs come from oracle.detinit (hash-based, framework
independent), so fixtures store only outputs: losses, checksums, sampled
entries and per-parameter gradient statistics.

Usage:  python tests/golden/make_golden.py          (blocks, B=2/T=44, B=1/T=252)
        python tests/golden/make_golden.py bench    (B=32/T=252, the benchmarked config)
        python tests/golden/make_golden.py t860     (B=2/T=860, the reference's own training
                                                     chunk, and B=2/T=100, an off-grid length)
        python tests/golden/make_golden.py b16t860  (B=16/T=860: the reference's default batch,
                                                     train.py:219, on that chunk)
"""
import os
import sys
import zlib

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, "/root/reference/model")

import model as ref  # noqa: E402  (the reference model/model.py)

from oracle import detinit  # noqa: E402

torch.set_num_threads(8)
N_SAMPLE = 16


def sample_idx(name, n, k=N_SAMPLE):
    return detinit.randint("sample:" + name, (k,), 0, n).astype(np.int64)


def load_det(module, seed=0):
    sd = {}
    for n, p in module.named_parameters():
        sd[n] = torch.from_numpy(detinit.param_value(n, tuple(p.shape), seed))
    module.load_state_dict(sd, strict=True)


def grad_stats(module, prefix="g"):
    out = {}
    names = []
    for n, p in module.named_parameters():
        names.append(n)
        if p.grad is None:
            out[f"{prefix}none:{n}"] = np.array(1)
            continue
        g = p.grad.detach().double().numpy().ravel()
        out[f"{prefix}stat:{n}"] = np.array([g.sum(), np.abs(g).sum(), (g * g).sum()])
        idx = sample_idx(n, g.size)
        out[f"{prefix}idx:{n}"] = idx
        out[f"{prefix}val:{n}"] = g[idx].astype(np.float32)
    return out, names


def out_len(T):
    """PerformanceNet's output length (model.py:229-232: the up-kernels 6/4/3/2 give
    16 * floor(T / 16) + 12), T itself only when T = 12 (mod 16)."""
    return 16 * (T // 16) + 12


def _run(net, B, T, dtype):
    xm, xa, cd, tg = (torch.from_numpy(a).to(dtype) for a in detinit.model_inputs(B, T))
    if out_len(T) != T:
        # off-grid length: the reference's L1Loss (train.py:132) needs a target of the output's
        # length, so the target is drawn at that length (detinit.offgrid_target)
        tg = torch.from_numpy(detinit.offgrid_target(B, out_len(T))).to(dtype)
    net.zero_grad(set_to_none=True)
    y = net(xm, xa, cd)
    loss = nn.L1Loss()(y, tg)
    loss.backward()
    return y, loss, (xm, xa, cd, tg)


def full_model(B, T, fname, adam=True):
    """fp32 run (what the reference computes) plus an fp64 run of the same reference model
    (the numerical truth). The fp32-vs-fp64 gap of the reference itself calibrates the parity
    tolerance: L1's sign(), LeakyReLU/ReLU kinks and maxpool argmax make this network's
    gradients ill-conditioned (per-parameter L2 gaps of 1-13% between fp32 and fp64)."""
    torch.manual_seed(0)
    net = ref.PerformanceNet()
    load_det(net)
    net.eval()  # dropout off; InstanceNorm has no running stats so only dropout differs
    net64 = ref.PerformanceNet()
    load_det(net64)
    net64.double().eval()
    y, loss, _ = _run(net, B, T, torch.float32)
    y64, loss64, _ = _run(net64, B, T, torch.float64)
    yv = y.detach().double().numpy().ravel()
    yv64 = y64.detach().numpy().ravel()
    oidx = detinit.randint("outidx", (512,), 0, yv.size).astype(np.int64)
    out = {
        "B": np.array(B), "T": np.array(T),
        "loss": np.array(loss.item(), dtype=np.float64),
        "loss64": np.array(loss64.item(), dtype=np.float64),
        "out_stat": np.array([yv.sum(), np.abs(yv).sum(), (yv * yv).sum()]),
        "out_idx": oidx, "out_val": yv[oidx].astype(np.float32), "out_val64": yv64[oidx],
        "out_shape": np.array(y.shape),
    }
    names = []
    p64 = dict(net64.named_parameters())
    for n, p in net.named_parameters():
        names.append(n)
        if p.grad is None:
            out[f"gnone:{n}"] = np.array(1)
            continue
        g = p.grad.detach().double().numpy().ravel()
        g64 = p64[n].grad.detach().numpy().ravel()
        idx = sample_idx(n, g.size, 256)
        out[f"gidx:{n}"] = idx
        out[f"gval:{n}"] = g[idx].astype(np.float32)
        out[f"gval64:{n}"] = g64[idx]
        out[f"gstat:{n}"] = np.array([g.sum(), np.abs(g).sum(), (g * g).sum(),
                                      np.linalg.norm(g - g64), np.linalg.norm(g64)])
    out["param_names"] = np.array(names)
    if adam:
        opt = torch.optim.Adam(net.parameters(), lr=1e-3)
        opt.step()
        for n, p in net.named_parameters():
            if p.grad is None:
                continue
            out[f"adam:{n}"] = p.detach().numpy().ravel()[out[f"gidx:{n}"]].astype(np.float32)
        opt.zero_grad()
        _, loss2, _ = _run(net, B, T, torch.float32)
        opt.step()
        out["loss2"] = np.array(loss2.item(), dtype=np.float64)
        opt64 = torch.optim.Adam(net64.parameters(), lr=1e-3)
        opt64.step()  # net64 still holds its step-0 gradients
        _, loss2_64, _ = _run(net64, B, T, torch.float64)
        out["loss2_64"] = np.array(loss2_64.item(), dtype=np.float64)
        for n, p in net.named_parameters():
            if p.grad is None:
                continue
            out[f"adam2:{n}"] = p.detach().numpy().ravel()[out[f"gidx:{n}"]].astype(np.float32)
    np.savez_compressed(os.path.join(HERE, fname), **out)
    print("wrote", fname, "loss", loss.item(), "loss64", loss64.item())


def full_model_lowmem(B, T, fname):
    """full_model without Adam for a large batch (the benchmarked B=32, T=252): the fp32 and
    fp64 reference runs happen one after the other so only one network is alive at a time."""
    res = {}
    for dtype in (torch.float32, torch.float64):
        torch.manual_seed(0)
        net = ref.PerformanceNet()
        load_det(net)
        net = net.to(dtype).eval()
        y, loss, _ = _run(net, B, T, dtype)
        res[dtype] = (y.detach().double().numpy().ravel(), loss.item(),
                      {n: (p.grad.detach().double().numpy().ravel() if p.grad is not None else None)
                       for n, p in net.named_parameters()})
        del net, y
    yv, loss, g32 = res[torch.float32]
    yv64, loss64, g64s = res[torch.float64]
    oidx = detinit.randint("outidx", (512,), 0, yv.size).astype(np.int64)
    out = {"B": np.array(B), "T": np.array(T), "loss": np.array(loss, dtype=np.float64),
           "loss64": np.array(loss64, dtype=np.float64),
           "out_stat": np.array([yv.sum(), np.abs(yv).sum(), (yv * yv).sum()]),
           "out_idx": oidx, "out_val": yv[oidx].astype(np.float32), "out_val64": yv64[oidx],
           "out_shape": np.array([B, 1025, out_len(T)])}
    names = list(g32)
    for n in names:
        g, g64 = g32[n], g64s[n]
        if g is None:
            out[f"gnone:{n}"] = np.array(1)
            continue
        idx = sample_idx(n, g.size, 256)
        out[f"gidx:{n}"] = idx
        out[f"gval:{n}"] = g[idx].astype(np.float32)
        out[f"gval64:{n}"] = g64[idx]
        out[f"gstat:{n}"] = np.array([g.sum(), np.abs(g).sum(), (g * g).sum(),
                                      np.linalg.norm(g - g64), np.linalg.norm(g64)])
    out["param_names"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, fname), **out)
    print("wrote", fname, "loss", loss, "loss64", loss64)


def blocks():
    """Small-shape per-block vectors (full tensors) for DownConv/UpConv/DenseConcat/MBR/crop."""
    out = {}

    def t(name, shape, lo=-1, hi=1):
        return torch.from_numpy(detinit.uniform(name, shape, lo, hi))

    # DownConv (model.py:34-53), pooled and unpooled, odd length to exercise floor pooling
    for pool in (True, False):
        m = ref.DownConv(5, 7, block_id=0, pooling=pool)
        load_det(m, seed=3)
        x = t("dc_x", (2, 5, 13)).requires_grad_(True)
        y, before = m(x)
        r1, r2 = t("dc_r1", tuple(y.shape)), t("dc_r2", tuple(before.shape))
        ((y * r1).sum() + (before * r2).sum()).backward()
        k = f"downconv_pool{int(pool)}"
        out[k + ":x"] = x.detach().numpy()
        out[k + ":y"] = y.detach().numpy()
        out[k + ":before"] = before.detach().numpy()
        out[k + ":dx"] = x.grad.numpy()
        for n, p in m.named_parameters():
            out[k + ":d:" + n] = p.grad.numpy()

    # UpConv (model.py:56-90) for every up-kernel and skip offsets around the upsampled length
    for (kk, cond) in ((6, 3), (4, 2), (3, 0), (2, 0)):
        for dskip in (-3, -2, -1, 0, 1, 2, 3):
            m = ref.UpConv(6, 4, 3, cond, block_id=5, upconv_kernel=kk)
            load_det(m, seed=5)
            Tin = 9
            Lu = (Tin - 1) * 2 - 2 + kk
            dec = t(f"uc_dec{kk}", (2, 6, Tin)).requires_grad_(True)
            res = t(f"uc_res{kk}{dskip}", (2, 3, Lu + dskip)).requires_grad_(True)
            c = t(f"uc_c{kk}{dskip}", (2, cond, Lu - 1)).requires_grad_(True) if cond else None
            y = m(res, dec, c)
            r = t(f"uc_r{kk}{dskip}", tuple(y.shape))
            (y * r).sum().backward()
            k = f"upconv_k{kk}_d{dskip}"
            out[k + ":dec"] = dec.detach().numpy()
            out[k + ":res"] = res.detach().numpy()
            if cond:
                out[k + ":cond"] = c.detach().numpy()
                out[k + ":dcond"] = c.grad.numpy()
            out[k + ":y"] = y.detach().numpy()
            out[k + ":ddec"] = dec.grad.numpy()
            out[k + ":dres"] = res.grad.numpy()
            for n, p in m.named_parameters():
                out[k + ":d:" + n] = p.grad.numpy()

    # DenseConcat (model.py:93-108), eval mode (dropout identity)
    m = ref.DenseConcat(5 + 3, 6, 5)
    load_det(m, seed=7)
    m.eval()
    mid = t("dn_midi", (2, 5, 11)).requires_grad_(True)
    aud = t("dn_audio", (2, 3, 11)).requires_grad_(True)
    y = m(mid, aud)
    r = t("dn_r", tuple(y.shape))
    (y * r).sum().backward()
    out["dense:midi"], out["dense:audio"] = mid.detach().numpy(), aud.detach().numpy()
    out["dense:y"], out["dense:dmidi"], out["dense:daudio"] = (
        y.detach().numpy(), mid.grad.numpy(), aud.grad.numpy())
    for n, p in m.named_parameters():
        out["dense:d:" + n] = p.grad.numpy()

    # MBRBlock (model.py:143-174): returns exactly 2*x, convs receive no gradient
    m = ref.MBRBlock(16, 4)
    load_det(m, seed=9)
    x = t("mbr_x", (2, 16, 10)).requires_grad_(True)
    y = m(x)
    y.sum().backward()
    out["mbr:x"], out["mbr:y"] = x.detach().numpy(), y.detach().numpy()
    out["mbr:conv_grads_none"] = np.array(all(p.grad is None for p in m.parameters()))

    # Onset_Offset_Encoder (model.py:111-141)
    m = ref.Onset_Offset_Encoder(depth=3, start_channels=4)
    load_det(m, seed=11)
    x = t("oe_x", (2, 4, 44)).requires_grad_(True)
    conds = m(x)
    (sum((c * t(f"oe_r{i}", tuple(c.shape))).sum() for i, c in enumerate(conds))).backward()
    out["onset:x"] = x.detach().numpy()
    out["onset:n"] = np.array(len(conds))
    for i, c in enumerate(conds):
        out[f"onset:c{i}"] = c.detach().numpy()
    out["onset:dx"] = x.grad.numpy()

    # crop_and_concat in isolation
    uc = ref.UpConv(2, 2, 2, 0, block_id=0)
    for d in range(-3, 4):
        up = t("cc_up", (1, 2, 10))
        byp = t(f"cc_b{d}", (1, 2, 10 + d))
        out[f"crop:d{d}:byp"] = byp.numpy()
        out[f"crop:d{d}:out"] = uc.crop_and_concat(up, byp).numpy()
    out["crop:up"] = t("cc_up", (1, 2, 10)).numpy()
    np.savez_compressed(os.path.join(HERE, "blocks.npz"), **out)
    print("wrote blocks.npz")


if __name__ == "__main__":
    if sys.argv[1:] == ["bench"]:  # the benchmarked configuration only (slow: ~minutes on CPU)
        full_model_lowmem(32, 252, "full_B32_T252.npz")
        sys.exit(0)
    if sys.argv[1:] == ["t860"]:  # the reference's training chunk (preprocess.py:42,66) + off-grid T
        full_model_lowmem(2, 860, "full_B2_T860.npz")
        full_model_lowmem(2, 100, "full_B2_T100.npz")
        sys.exit(0)
    if sys.argv[1:] == ["b16t860"]:  # the reference's default batch (train.py:219) on that chunk
        full_model_lowmem(16, 860, "full_B16_T860.npz")
        sys.exit(0)
    blocks()
    full_model(2, 44, "full_B2_T44.npz")
    full_model(1, 252, "full_B1_T252.npz", adam=False)
    print("crc", zlib.crc32(open(os.path.join(HERE, "blocks.npz"), "rb").read()))
