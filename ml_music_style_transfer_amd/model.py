"""Drop-in PerformanceNet (reference model/model.py) running on libmst_hip kernels.

Same constructor arguments, module tree, parameter names/shapes/order and
state_dict keys as the reference, so reference checkpoints
(`torch.save({'state_dict': model.state_dict(), ...})`, train.py:204) load
with `load_state_dict` (inference.py:78). The forward math is executed by the
hand-written gfx950 kernels (engine.py); there is no CPU path — a model on CPU
raises on forward.

Blocks (DownConv, UpConv, DenseConcat, Onset_Offset_Encoder, MBRBlock) are
usable standalone through per-block autograd functions; PerformanceNet runs
the whole network as one fused program (engine.PerformanceNetFunction) with
its trainable parameters stored in one flat device buffer (and gradients in a
parallel flat buffer) so Adam and the data-parallel all-reduce each touch one
contiguous range.
"""
import os
import weakref

import torch
import torch.nn as nn
from torch.nn import init

from . import engine as E
from . import kernels as K


def conv1x3(in_channels, out_channels, stride=1, padding=1, bias=True, groups=1):
    """model.py:14-22."""
    return nn.Conv1d(in_channels, out_channels, kernel_size=3, stride=stride, padding=padding,
                     bias=bias, groups=groups)


def upconv1x2(in_channels, out_channels, kernel):
    """model.py:24-31."""
    return nn.ConvTranspose1d(in_channels, out_channels, kernel_size=kernel, stride=2, padding=1)


def slot_view(buf, p):
    """View of a flat-buffer slot with p's shape. 3-D conv weights (Conv1d (Cout, Cin, k),
    ConvTranspose1d (Cin, Cout, k)) are stored tap-major, i.e. as (d0, k, d1) permuted back
    to (d0, d1, k): the GEMM loaders then read channel-contiguous rows (float4 along K for
    the forward of Conv1d, along M for its input gradient)."""
    if p.dim() == 3:
        d0, d1, k = p.shape
        return buf.view(d0, k, d1).permute(0, 2, 1)
    return buf.view_as(p)


# The weight-gradient GEMMs run on a side stream (engine.GradSink), concurrently with the
# input-gradient GEMMs. With the fp32-MFMA GEMMs it gained 0.6 % (profiles/r02/
# bench_m7_wgrad_stream.txt); with the shorter bf16x6 GEMMs 2.2 % (44.71 -> 43.84 ms/step,
# profiles/r02/bench_m15_*.json), so it is on by default. MST_WGRAD_STREAM=0 turns it off;
# set_wgrad_stream(False) does too (bench.py's per-launch timing leg: overlapping kernels
# would make per-launch times meaningless). Stream capture (graphs.py) always runs serially.
_WGRAD_STREAM = os.environ.get("MST_WGRAD_STREAM", "1") == "1"
# the last N backward blocks' weight gradients on the main stream (engine.GradSink); A/B knob
_WGRAD_MAIN_TAIL = int(os.environ.get("MST_WGRAD_MAIN_TAIL", "6"))
# the audio encoder on a second stream beside the MIDI / onset encoders (engine.network_fwd /
# network_bwd); MST_ENC_STREAM=0 runs the encoders one after the other
_ENC_STREAM = os.environ.get("MST_ENC_STREAM", "1") == "1"


def set_wgrad_stream(on):
    """Enable / disable the side stream for weight-gradient GEMMs (process-wide)."""
    global _WGRAD_STREAM
    _WGRAD_STREAM = bool(on)


def set_enc_stream(on):
    """Enable / disable the encoder stream (process-wide; bench.py's per-launch timing leg
    serialises it with the weight-gradient stream)."""
    global _ENC_STREAM
    _ENC_STREAM = bool(on)


def _require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("ml_music_style_transfer_amd runs on the GPU only (HIP kernels); "
                               "move the module and inputs to 'cuda'")


# ----------------------------------------------------------- per-block autograd
class _DownConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, W1, b1, W2, b2):
        out, before, saved = E.downconv_fwd(W1, b1, W2, b2, x.contiguous(), mod.pooling)
        ctx.saved = saved
        ctx.params = (W1, b1, W2, b2)
        ctx.pooling = mod.pooling
        return out, before

    @staticmethod
    def backward(ctx, d_out, d_before):
        d_out = d_out.contiguous() if d_out is not None else None
        d_before = d_before.contiguous() if d_before is not None else None
        if ctx.pooling:
            dx = E.downconv_bwd(ctx.params, ctx.saved, E.GradSink(), d_before=d_before,
                                d_pool0=d_out, need_dx=True)
        else:
            d = d_before if d_out is None else (d_out if d_before is None else d_out + d_before)
            dx = E.downconv_bwd(ctx.params, ctx.saved, E.GradSink(), d_before=d, need_dx=True)
        return None, dx, None, None, None, None


class _DenseConcatFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, drop_p, seed, midi, audio, W1, b1, W2, b2):
        h2, saved = E.dense_fwd(W1, b1, W2, b2, midi.contiguous(), audio.contiguous(), drop_p, seed)
        ctx.saved = saved
        ctx.params = (W1, b1, W2, b2)
        return h2

    @staticmethod
    def backward(ctx, d_h2):
        d_midi, d_audio = E.dense_bwd(ctx.params, ctx.saved, E.GradSink(), d_h2.contiguous())
        return None, None, d_midi, d_audio, None, None, None, None


class _UpConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, res, dec, cond, Wu, bu, W1, b1, W2, b2):
        w, saved = E.upconv_fwd(Wu, bu, W1, b1, W2, b2, res.contiguous(), dec.contiguous(),
                                cond.contiguous() if cond is not None else None)
        ctx.saved = saved
        ctx.params = (Wu, bu, W1, b1, W2, b2)
        ctx.has_cond = cond is not None
        return w

    @staticmethod
    def backward(ctx, d_w):
        d_res, d_dec, d_cond = E.upconv_bwd(ctx.params, ctx.saved, E.GradSink(), d_w.contiguous())
        return (d_res, d_dec, d_cond if ctx.has_cond else None) + (None,) * 6


class _ScaleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, s):
        y = x.contiguous().clone()
        K.scale_(y, s)
        ctx.s = s
        return y

    @staticmethod
    def backward(ctx, g):
        d = g.contiguous().clone()
        K.scale_(d, ctx.s)
        return d, None


# -------------------------------------------------------------------- blocks
class DownConv(nn.Module):
    """model.py:34-53."""

    def __init__(self, in_channels, out_channels, block_id, pooling=True):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.pooling = pooling
        self.activation = nn.LeakyReLU(0.01)
        self.conv1 = conv1x3(self.in_channels, self.out_channels)
        self.conv1_BN = nn.InstanceNorm1d(self.out_channels)
        self.conv2 = conv1x3(self.out_channels, self.out_channels)
        self.conv2_BN = nn.InstanceNorm1d(self.out_channels)
        self.pool = nn.MaxPool1d(kernel_size=2, stride=2)

    def forward(self, x):
        _require_cuda(x)
        return _DownConvFn.apply(self, x, self.conv1.weight, self.conv1.bias, self.conv2.weight,
                                 self.conv2.bias)


class UpConv(nn.Module):
    """model.py:56-90."""

    def __init__(self, in_channels, out_channels, skip_channels, cond_channels, block_id,
                 activation=None, upconv_kernel=2):
        super().__init__()
        self.skip_channels = skip_channels
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.cond_channels = cond_channels
        self.activation = activation if activation is not None else nn.LeakyReLU(0.01)
        self.upconv = upconv1x2(self.in_channels, self.out_channels, kernel=upconv_kernel)
        self.upconv_BN = nn.InstanceNorm1d(self.out_channels)
        self.conv1 = conv1x3(self.skip_channels + self.out_channels, self.out_channels)
        self.conv1_BN = nn.InstanceNorm1d(self.out_channels)
        self.conv2 = conv1x3(self.out_channels + self.cond_channels, self.out_channels)
        self.conv2_BN = nn.InstanceNorm1d(self.out_channels)

    @staticmethod
    def crop_and_concat(upsampled, bypass):
        """model.py:71-78 on the device: cat(upsampled, bypass shifted by (Lb-Lu)//2)."""
        Lu = upsampled.shape[2]
        c = E.crop_offset(bypass.shape[2], Lu)
        out = torch.zeros(upsampled.shape[0], bypass.shape[1], Lu, device=bypass.device,
                          dtype=bypass.dtype)
        lo, hi = max(0, -c), min(Lu, bypass.shape[2] - c)
        if hi > lo:
            out[:, :, lo:hi] = bypass[:, :, lo + c:hi + c]
        return torch.cat((upsampled, out), 1)

    def forward(self, res, dec, cond):
        _require_cuda(res, dec, cond)
        return _UpConvFn.apply(res, dec, cond if self.cond_channels else None, self.upconv.weight,
                               self.upconv.bias, self.conv1.weight, self.conv1.bias,
                               self.conv2.weight, self.conv2.bias)


class DenseConcat(nn.Module):
    """model.py:93-108."""

    def __init__(self, in_channels, intermediate_channels, out_channels):
        super().__init__()
        self.fc1 = nn.Linear(in_channels, intermediate_channels)
        self.fc2 = nn.Linear(intermediate_channels, out_channels)
        self.dropout = nn.Dropout(p=0.2)
        self._seed = 0

    def forward(self, midi_embed, audio_embed):
        _require_cuda(midi_embed, audio_embed)
        p = self.dropout.p if self.training else 0.0
        self._seed += 2
        return _DenseConcatFn.apply(p, self._seed, midi_embed, audio_embed, self.fc1.weight,
                                    self.fc1.bias, self.fc2.weight, self.fc2.bias)


class Onset_Offset_Encoder(nn.Module):
    """model.py:111-141."""

    def __init__(self, depth=3, start_channels=128):
        super().__init__()
        self.start_channels = start_channels
        self.depth = depth
        down_convs = []
        outs = start_channels
        for i in range(self.depth):
            ins = self.start_channels if i == 0 else outs
            outs = self.start_channels * (2 ** (i + 1))
            down_convs.append(DownConv(ins, outs, pooling=True, block_id=i + 9))
        self.down_convs = nn.ModuleList(down_convs)
        self.reset_params()

    @staticmethod
    def weight_init(m):
        if isinstance(m, nn.Conv1d):
            init.xavier_normal_(m.weight)
            init.constant_(m.bias, 0)

    def reset_params(self):
        for m in self.modules():
            self.weight_init(m)

    def forward(self, x):
        condition_tensors = []
        for i, module in enumerate(self.down_convs):
            x, _ = module(x)
            if i > self.depth - 3:
                condition_tensors.append(x)
        return condition_tensors


class MBRBlock(nn.Module):
    """model.py:143-174. The reference's per-band residual is discarded
    (`torch.add(bands[i],1,t)` result unused, :172), so the block returns 2*x and its
    convolutions never receive gradients; the parameters are kept for state_dict parity."""

    def __init__(self, in_channels, num_of_band):
        super().__init__()
        self.in_dim = in_channels
        self.num_of_band = num_of_band
        self.activation = nn.LeakyReLU(0.01)
        self.band_dim = self.in_dim // self.num_of_band
        bd = self.band_dim
        self.conv_list1 = nn.ModuleList([nn.Conv1d(bd, bd, kernel_size=3, padding=1)
                                         for _ in range(num_of_band)])
        self.conv_list2 = nn.ModuleList([nn.Conv1d(bd, bd, kernel_size=3, padding=1)
                                         for _ in range(num_of_band)])
        self.bn_list1 = nn.ModuleList([nn.InstanceNorm1d(bd) for _ in range(num_of_band)])
        self.bn_list2 = nn.ModuleList([nn.InstanceNorm1d(bd) for _ in range(num_of_band)])

    def forward(self, x):
        _require_cuda(x)
        return _ScaleFn.apply(x, 2.0)


class PerformanceNet(nn.Module):
    """model.py:177-300."""

    def __init__(self, depth=5, start_channels=128, start_audio_channels=1025):
        super().__init__()
        self.depth = depth
        self.start_channels = start_channels
        self.start_audio_channels = start_audio_channels
        self.construct_layers()
        self.reset_params()
        self._flat = None
        self._seed = 0x5EED

    def construct_layers(self):
        outs_channel_list_midi = []
        down_convs = []
        outs = self.start_channels
        for i in range(self.depth):
            ins = self.start_channels if i == 0 else outs
            outs = self.start_channels * (2 ** (i + 1))
            outs_channel_list_midi.append(outs)
            down_convs.append(DownConv(ins, outs, pooling=i < self.depth - 1, block_id=i))
        self.down_convs = nn.ModuleList(down_convs)

        outs_channel_list_audio = [int(1024 * 1.5), 2048, int(2048 * 1.5), 4096, int(4096 * 1.5)]
        down_convs_audio = []
        for i in range(self.depth):
            ins = self.start_audio_channels if i == 0 else outs
            outs = outs_channel_list_audio[i]
            down_convs_audio.append(DownConv(ins, outs, pooling=i < self.depth - 1, block_id=i))
        self.down_convs_audio = nn.ModuleList(down_convs_audio)

        dense_concats = []
        for i in range(self.depth):
            out_midi = outs_channel_list_midi[-(i + 1)]
            out_audio = outs_channel_list_audio[-(i + 1)]
            dense_concats.append(DenseConcat(out_midi + out_audio, int(out_midi * 1.5), out_midi))
        self.dense_concats = nn.ModuleList(dense_concats)

        self.up_convs = nn.ModuleList([
            UpConv(4096, 2048, 2048, 1024, block_id=5, upconv_kernel=6),
            UpConv(2048, 1024, 1024, 512, block_id=6, upconv_kernel=4),
            UpConv(1024, 1024, 512, 0, block_id=7, upconv_kernel=3),
            UpConv(1024, 1024, 256, 0, block_id=8),
        ])

        self.MBRBlock1 = MBRBlock(1024, 2)
        self.MBRBlock2 = MBRBlock(1024, 4)
        self.MBRBlock3 = MBRBlock(1024, 8)
        self.MBRBlock4 = MBRBlock(1024, 16)

        self.lastconv = nn.ConvTranspose1d(1024, 1025, kernel_size=3, stride=1, padding=1)
        self.lrelu = nn.LeakyReLU(0.01)

        self.onset_offset_encoder = Onset_Offset_Encoder()

    @staticmethod
    def weight_init(m):
        if isinstance(m, (nn.Conv1d, nn.ConvTranspose1d)):
            init.xavier_normal_(m.weight)
            init.constant_(m.bias, 0)

    def reset_params(self):
        for m in self.modules():
            self.weight_init(m)

    # ------------------------------------------------------------ flat storage
    def _trainable_named(self):
        """Parameters that receive gradients (all but the dead MBR convs), reference order."""
        return [(n, p) for n, p in self.named_parameters() if not n.startswith("MBRBlock")]

    def _flat_params_list(self):
        return [p for _, p in self._trainable_named()]

    def _param_dict(self):
        return dict(self._trainable_named())

    def _flat_ok(self):
        f = self._flat
        if f is None:
            return False
        params = self._flat_params_list()
        if len(params) != len(f["offsets"]) or params[0].device != f["param"].device:
            return False
        base = f["param"].data_ptr()
        for p, off in zip(params, f["offsets"]):
            if p.data_ptr() != base + 4 * off:
                return False
        return True

    def flatten_parameters_(self):
        """Move trainable parameters into one contiguous device buffer (16-B aligned slots)."""
        named = self._trainable_named()
        params = [p for _, p in named]
        dev = params[0].device
        # Slots are laid out in the order backward produces the gradients (lastconv first,
        # the input-side encoder levels last) so data-parallel buckets fill front to back.
        rank = {n: i for i, n in enumerate(E.backward_param_order(self.depth))}
        order = sorted(range(len(named)), key=lambda i: (rank.get(named[i][0], len(rank)), i))
        offsets, off = [0] * len(params), 0
        for i in order:
            offsets[i] = off
            off += (params[i].numel() + 3) // 4 * 4
        flat = torch.zeros(off, device=dev, dtype=torch.float32)
        grad = torch.zeros(off, device=dev, dtype=torch.float32)
        with torch.no_grad():
            for p, o in zip(params, offsets):
                dst = slot_view(flat[o:o + p.numel()], p)
                dst.copy_(p.data)
                p.data = dst
                if p.grad is not None:
                    g = slot_view(grad[o:o + p.numel()], p)
                    g.copy_(p.grad)
                    p.grad = g
        me = weakref.ref(self)
        for p in params:
            p._mst_flat_owner = me
        self._flat = {"param": flat, "grad": grad, "offsets": offsets, "numel": off,
                      "index": {id(p): (o, p.numel()) for p, o in zip(params, offsets)}}
        return self._flat

    def flat_buffers(self):
        """(flat params, flat grads, total length) of the trainable parameters."""
        if not self._flat_ok():
            self.flatten_parameters_()
        f = self._flat
        return f["param"], f["grad"], f["numel"]

    def _grad_sink(self, on_ready=None):
        f = self._flat

        def flat_grad_of(p):
            ent = f["index"].get(id(p)) if f is not None else None
            if ent is None:
                return None
            o, n = ent
            return slot_view(f["grad"][o:o + n], p)
        side = None
        if _WGRAD_STREAM and not torch.cuda.is_current_stream_capturing():
            dev = f["grad"].device if f is not None else torch.device("cuda", torch.cuda.current_device())
            side = self.__dict__.get("_mst_side")
            if side is None or side.device != dev:
                side = self.__dict__["_mst_side"] = torch.cuda.Stream(device=dev)
        return E.GradSink(flat_grad_of, on_ready, side, _WGRAD_MAIN_TAIL,
                          self.__dict__.get("_mst_bwd_blocks"))

    def _enc_stream(self):
        """The audio encoder's stream (None: serial; always under stream capture)."""
        if not _ENC_STREAM or torch.cuda.is_current_stream_capturing():
            return None
        dev = torch.device("cuda", torch.cuda.current_device())
        s = self.__dict__.get("_mst_enc")
        if s is None or s.device != dev:
            s = self.__dict__["_mst_enc"] = torch.cuda.Stream(device=dev)
        return s

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._flat = None
        params = self._flat_params_list()
        if params and params[0].is_cuda:
            self.flatten_parameters_()
        return out

    def _dropout_p(self):
        return self.dense_concats[0].dropout.p

    def _next_seed(self):
        self._seed += 1
        return (self._seed * 0x9E3779B1) & 0xFFFFFFFFFFFF

    # ----------------------------------------------------------------- forward
    def forward(self, x_midi, x_audio, cond):
        """model.py:262-300: (B,128,T) piano roll, (B,1025,T) spectrogram, (B,128,T) onoff
        -> (B,1025,T). T must be >= 44 and T % 16 == 12 for the output to match T
        (the reference's up-kernel geometry)."""
        _require_cuda(x_midi, x_audio, cond)
        if not self._flat_ok():
            self.flatten_parameters_()
        return E.PerformanceNetFunction.apply(self, x_midi, x_audio, cond, *self._flat_params_list())
