"""The multi-scale spectral loss as a TRAINING loss (README.md:23, the
engel_loss stub at model/train.py:119-123): one PerformanceNet step whose loss is
spectral.spectrogram_mss_loss on the model's log-power output, on the HIP path (fused render
kernel, iSTFT with its adjoint, mss kernels, the model's backward) against a torch float64
restatement of the same pipeline on the CPU (oracle/model_ref.py's functional PerformanceNet,
torch.istft, torch.stft), with the phase held as the loss holds it.

Tolerances: loss 1e-4 relative (north_star); the gradient at the model output (the render /
iSTFT / loss chain evaluated in float64 at this model output) within max(2 x torch fp32's gap,
2 %) rel L2 (the MSS's 1/(S + eps) factor, test_istft_grad.py), and every sampled weight gradient
within max(4 x the torch fp32 CPU gap, 2 %) rel L2 of the float64 step. The loss is this build's
definition (the reference has only the stub): parity unpinned against the reference.
"""
import numpy as np
import pytest
import torch

from oracle import detinit
from oracle import model_ref as R

pytestmark = pytest.mark.gpu
N_FFT, HOP = 2048, 256


def _target_audio(B, L):
    import bench
    x, _ = bench.synth_clips(B, 4711, L=L)
    rng = np.random.default_rng(5)
    return (x + 1e-3 * rng.standard_normal(x.shape)).astype(np.float32)  # no exact silence


def _torch_mss(y, yt, sizes):
    tot = 0
    for n in sizes:
        w = torch.hann_window(n, periodic=True, dtype=y.dtype)
        a = torch.stft(y, n, n // 4, window=w, center=True, pad_mode="reflect", return_complex=True).abs()
        b = torch.stft(yt, n, n // 4, window=w, center=True, pad_mode="reflect", return_complex=True).abs()
        tot = tot + (a - b).abs().mean() + (torch.log(a + 1e-7) - torch.log(b + 1e-7)).abs().mean()
    return tot


def _cpu_step(dtype, P, yt, B, T, sizes, S_in=None):
    """The restated step in `dtype` on the CPU: forward, render with P's phase, istft, MSS, grads.
    With S_in the chain starts at that model output (no forward; parameter grads None)."""
    p = {k: v.to(dtype).requires_grad_(True) for k, v in R.det_params().items()} if S_in is None else {}
    if S_in is None:
        xm, xa, cd, _ = (torch.from_numpy(a).to(dtype) for a in detinit.model_inputs(B, T))
        S = R.forward(p, xm, xa, cd)
        S.retain_grad()
    else:
        S = S_in.to(dtype).clone().requires_grad_(True)
    U = P / P.abs().clamp_min(1e-300)
    U = torch.where(P.abs() > 0, U, torch.ones_like(U)).to(torch.complex128 if dtype == torch.float64
                                                            else torch.complex64)
    M = torch.expm1(S.clamp(0, 20)).sqrt()
    X = M * U.transpose(1, 2)  # (B, F, T)
    win = torch.hann_window(N_FFT, periodic=True, dtype=dtype)
    y = torch.istft(X, N_FFT, HOP, window=win, center=True, length=HOP * (T - 1))
    loss = _torch_mss(y, yt.to(dtype), sizes)
    loss.backward()
    return loss.item(), S.grad, {k: v.grad for k, v in p.items()}


@pytest.mark.parametrize("phase", ["target", "griffinlim"])
def test_performancenet_step_with_mss_loss(cuda, phase):
    from ml_music_style_transfer_amd import spectral
    from ml_music_style_transfer_amd.model import PerformanceNet
    from ml_music_style_transfer_amd.train import make_optimizer
    B, T = 1, 44
    L = HOP * (T - 1)
    sizes = spectral.MSS_SIZES
    net = PerformanceNet()
    net.load_state_dict({n: torch.from_numpy(detinit.param_value(n, tuple(q.shape)))
                         for n, q in net.named_parameters()})
    net = net.to(cuda).eval()
    xm, xa, cd, _ = (torch.from_numpy(a).to(cuda) for a in detinit.model_inputs(B, T))
    yt = torch.from_numpy(_target_audio(B, L)).to(cuda)
    S = net(xm, xa, cd)
    S.retain_grad()
    loss = spectral.spectrogram_mss_loss(S, yt, phase=phase, gl_iters=4)
    loss.backward()
    # the held spectrum the loss used, recomputed the same way (deterministic) for the oracle
    with torch.no_grad():
        src = yt if phase == "target" else spectral.griffinlim(S.detach(), n_iter=4, init=None,
                                                               from_logpow=True)
        P = spectral.stft_complex(src).cpu().to(torch.complex128)  # (B, T, F)
    l64, _, g64 = _cpu_step(torch.float64, P, yt.cpu().double(), B, T, sizes)
    l32, _, g32 = _cpu_step(torch.float32, P, yt.cpu(), B, T, sizes)
    assert abs(loss.item() - l64) <= 1e-4 * abs(l64), (loss.item(), l64, l32)
    # the render / iSTFT / loss chain alone, in float64 at OUR model output: dM/dS = e^S / (2 M)
    # grows without bound as S -> 0+, so the chain is compared at the same S, not through two
    # forwards that round differently around S = 0
    Sg = S.detach().double().cpu()
    _, dS64, _ = _cpu_step(torch.float64, P, yt.cpu().double(), B, T, sizes, S_in=Sg)
    _, dS32, _ = _cpu_step(torch.float32, P, yt.cpu(), B, T, sizes, S_in=Sg)
    dS = S.grad.double().cpu()
    rel_out = ((dS - dS64).norm() / dS64.norm()).item()
    gap_out = ((dS32.double() - dS64).norm() / dS64.norm()).item()
    # bound: 4x torch fp32's own gap, floor 1e-4 (measured: 2.6e-5 / 2.9e-6 against torch fp32's
    # 9.6e-6 / 5.2e-6, profiles/r06/pytest_gpu_r6h.log; round 5 floored this at 2 %)
    assert rel_out <= max(4 * gap_out, 1e-4), (rel_out, gap_out)
    worst = []
    for n, q in net.named_parameters():
        if q.grad is None or g64.get(n) is None:
            continue
        idx = torch.from_numpy(detinit.randint("mss_sample:" + n, (256,), 0, q.numel()))
        ours = q.grad.detach().double().cpu().reshape(-1)[idx]
        r64 = g64[n].reshape(-1)[idx]
        r32 = g32[n].double().reshape(-1)[idx]
        den = r64.norm().item() + 1e-30
        e_ours, e_ref = (ours - r64).norm().item() / den, (r32 - r64).norm().item() / den
        if n.endswith(".bias") and not (n.startswith("dense_concats") or n == "lastconv.bias"):
            continue  # conv biases followed by InstanceNorm: exact gradient 0 (rounding noise only)
        worst.append((e_ours, e_ref, n))
        # 4x torch fp32's own gap for the parameter, floor 1e-3 (round 5: 2e-2); no parameter's
        # torch fp32 gap is below 2.5e-3 here (profiles/r06/pytest_gpu_mss_train_s6b.log), so the
        # floor binds nowhere: the bound is the reference-gap rule alone
        assert e_ours <= max(4 * e_ref, 1e-3), (n, e_ours, e_ref)
    opt = make_optimizer(net, lr=1e-3)
    opt.step()
    assert all(torch.isfinite(q).all() for q in net.parameters())
    worst.sort()
    floored = [w for w in worst if 4 * w[1] < 1e-3]
    print(f"phase={phase}: {len(floored)} of {len(worst)} parameters under the 1e-3 floor, the "
          f"largest of ours there {max((w[0] for w in floored), default=0):.2e}")
    print(f"phase={phase}: loss {loss.item():.6f} vs fp64 {l64:.6f} (fp32 CPU {l32:.6f}); "
          f"dL/dS rel L2 {rel_out:.2e} (torch fp32 {gap_out:.2e}); worst weight-gradient gaps (ours, torch fp32, name) {worst[-3:]}")


def test_train_loop_with_mss_loss(cuda):
    """train.train with make_loss('l1+mss') (the -loss flag of train.main): a short epoch on
    the synthetic dataset runs, every step finite, the epoch loss above the L1 part alone."""
    from ml_music_style_transfer_amd import train as TR
    from ml_music_style_transfer_amd.model import PerformanceNet
    torch.manual_seed(0)
    net = PerformanceNet().to(cuda)
    opt = TR.make_optimizer(net, lr=1e-4)
    ds = TR.SyntheticSpectrogramDataset(4, T=44, seed=3, device=cuda)
    loader = torch.utils.data.DataLoader(ds, batch_size=2)
    hist = []
    TR.train(net, 0, loader, opt, hist, log_every=0, loss_fn=TR.make_loss("l1+mss", gl_iters=2))
    assert len(hist) == 2 and all(np.isfinite(hist)), hist
    with pytest.raises(ValueError):
        TR.make_loss("bogus")
