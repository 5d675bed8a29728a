"""Forward/backward programs of PerformanceNet on libmst_hip.

Each reference block (model/model.py) is a pair of functions operating on raw
device tensors: `*_fwd` enqueues the block's kernels and returns its outputs
plus a saved-state tuple; `*_bwd` enqueues the backward kernels, writes weight
gradients straight into each parameter's `.grad` (a view of the model's flat
gradient buffer) and returns input gradients. The whole network forward is ONE
autograd node (`PerformanceNetFunction`), so backward runs this hand-scheduled
program instead of ~200 generic autograd nodes, and cross-block fusions are
possible:

  * torch.cat / crop_and_concat (model.py:71-78, 103) never materialise: GEMM
    loaders read two sources with time offsets, and dgrad epilogues split the
    concatenated input gradient back into its parts;
  * the maxpool gradient and the skip gradient of an encoder level are summed
    inside the InstanceNorm backward kernel (no accumulation pass), which also emits the
    per-(b, c) row sums of its output: the producing conv's bias gradient needs only a
    (B, C) reduction instead of another pass over dy;
  * MBRBlock x4 returns 16*x exactly (model.py:172 discards its residual sum),
    so its dead convolutions are skipped and the 16 folds into lastconv's GEMM
    (alpha) — output- and gradient-identical to the reference;
  * lastconv's LeakyReLU runs in the GEMM epilogue; DenseConcat's
    ReLU+Dropout backward is applied by the fc2-dgrad epilogue as a gate.

Gradient accumulation follows torch semantics: a parameter whose .grad is None
gets a fresh gradient (written, not added); otherwise the kernel adds into it.
"""
import torch

from . import _lib as L
from . import kernels as K
from . import ops as _ops  # noqa: F401  (registers torch.ops.mst.*)

LRELU = L.ACT_LRELU
RELU = L.ACT_RELU


def _e(shape, like):
    return torch.empty(shape, device=like.device, dtype=torch.float32)


class GradSink:
    """Where weight gradients go: p.grad if present (accumulate) else a fresh buffer.

    `on_ready(params)` (optional) is told, at each block boundary of the backward program,
    which parameters' gradient kernels have all been launched on the current stream; the
    data-parallel reducer (dp.OverlappedAllReduce) starts bucket all-reduces from it.

    Weight-gradient GEMMs are off the backward's critical path (the next layer needs only the
    input gradient), so with a side stream (`side`) they run there, concurrently with the
    input-gradient GEMMs and norm kernels of the main stream: a GEMM's trailing partial wave of
    workgroups no longer leaves the chip half idle. Tensors a side launch reads are recorded on
    the side stream (the caching allocator must not hand them out again before it is done). The
    block listeners run with the side stream current (after it has waited for the main stream),
    and the main stream waits for the side stream only at the end.
    `joined` is the event the main stream last waited on: it completes with the last side-stream
    launch (the side stream may still carry the caching allocator's free markers behind it,
    which are events, not work)."""

    def __init__(self, flat_grad_of=None, on_ready=None, side=None, main_tail=0, blocks=None):
        self.flat_grad_of = flat_grad_of or (lambda p: None)
        self.on_ready = on_ready
        self.side = side
        self._side_pending = False
        self._pending = []
        self.joined = None
        # the weight gradients of the last `main_tail` blocks (of `blocks` in the previous
        # backward) run on the main stream: once the main stream's input gradients are done the
        # side stream still holds a backlog, so both streams then carry weight gradients. At
        # least one block keeps its weight gradients on the side stream (so join() always has
        # the side stream's last launch to wait for).
        self.block = 0
        if blocks is not None and main_tail > 0 and blocks > 1:
            self._main_from = blocks - min(main_tail, blocks - 1)
        else:
            self._main_from = None
        self.home = torch.cuda.current_stream() if side is not None else None  # backward's main stream
        # streams that wrote gradients in this backward (the encoder stream writes some): with no
        # side stream the listeners issue from whichever stream is current at a block boundary,
        # so that stream first waits for the others (a bucket may span blocks of two streams)
        self._writers = []

    def target(self, p):
        if self.on_ready is not None and self.side is None:
            cur = torch.cuda.current_stream()
            if cur not in self._writers:
                self._writers.append(cur)
        self._pending.append(p)
        if p.grad is None:
            g = self.flat_grad_of(p)
            if g is None:
                g = torch.empty_like(p)
            p.grad = g
            return g, False
        return p.grad, True

    def wgrad(self, launch, *reads):
        """Run a weight-gradient launch (on the side stream when there is one; the tail blocks'
        on the backward's main stream, which is idle by then while the encoder stream still
        runs the audio encoder's backward)."""
        if self.side is None:
            launch()
            return
        cur = torch.cuda.current_stream()
        if self._main_from is not None and self.block >= self._main_from:
            if cur == self.home:
                launch()
                return
            self.home.wait_stream(cur)
            with torch.cuda.stream(self.home):
                launch()
            for t in reads:
                t.record_stream(self.home)
            return
        main = cur
        self.side.wait_stream(main)
        with torch.cuda.stream(self.side):
            launch()
        for t in reads:
            t.record_stream(self.side)
        self._side_pending = True

    def join(self):
        if self._side_pending:
            ev = torch.cuda.Event()
            ev.record(self.side)
            torch.cuda.current_stream().wait_event(ev)
            self.joined = ev
            self._side_pending = False

    def block_done(self):
        if self.on_ready is not None and self._pending:
            if self.side is not None:
                # the listeners issue from the weight-gradient stream, which first waits for the
                # main stream up to this point: their collectives / updates then follow both
                # streams' gradient kernels, and the main stream never waits for the weight
                # gradients inside backward (joining it here, as rounds 1-4 did, serialised the
                # two streams at every block whenever a DP reducer or BackwardAdam was attached)
                cur = torch.cuda.current_stream()
                self.side.wait_stream(cur)
                if cur != self.home:  # tail weight gradients may sit on the home stream
                    self.side.wait_stream(self.home)
                with torch.cuda.stream(self.side):
                    self.on_ready(self._pending)
            else:
                # a bucket completed here may hold gradients another stream wrote (the skip
                # levels' DenseConcat backward on the encoder stream): the listeners' collectives
                # and updates issue from the current stream, so it waits for those writers first
                cur = torch.cuda.current_stream()
                for s in self._writers:
                    if s != cur:
                        cur.wait_stream(s)
                self.on_ready(self._pending)
        self._pending = []
        self.block += 1


# ------------------------------------------------------------------ DownConv
def downconv_fwd(W1, b1, W2, b2, x, pool):
    """DownConv.forward (model.py:47-53). Returns (out, before_pool, saved)."""
    B, _, T = x.shape
    Cout = W1.shape[0]
    y1 = _e((B, Cout, T), x)
    K.conv3_fwd([(x, 0)], W1, b1, y1)
    a1, _, m1, r1 = K.in_lrelu_fwd(y1, False)
    y2 = _e((B, Cout, T), x)
    K.conv3_fwd([(a1, 0)], W2, b2, y2)
    a2, pooled, m2, r2 = K.in_lrelu_fwd(y2, pool)
    saved = (x, y1, m1, r1, a1, y2, m2, r2)
    return (pooled if pool else a2), a2, saved


def downconv_bwd(params, saved, sink, d_before=None, d_pool0=None, d_pool1=None, need_dx=True):
    W1, b1, W2, b2 = params
    x, y1, m1, r1, a1, y2, m2, r2 = saved
    dy2, rs2 = K.in_lrelu_bwd(y2, m2, r2, d_before, d_pool0, d_pool1, rowsum=True)
    g, acc = sink.target(W2)
    sink.wgrad(lambda: K.conv3_wgrad(dy2, [(a1, 0)], g, acc), dy2, a1)
    g, acc = sink.target(b2)
    K.bias_grad_rows(rs2, g, acc)
    da1 = torch.empty_like(a1)
    K.conv3_dgrad(dy2, W2, [(da1, 0, None, 1.0)])
    del dy2
    dy1, rs1 = K.in_lrelu_bwd(y1, m1, r1, da1, rowsum=True)
    del da1
    g, acc = sink.target(W1)
    sink.wgrad(lambda: K.conv3_wgrad(dy1, [(x, 0)], g, acc), dy1, x)
    g, acc = sink.target(b1)
    K.bias_grad_rows(rs1, g, acc)
    if not need_dx:
        return None
    dx = torch.empty_like(x)
    K.conv3_dgrad(dy1, W1, [(dx, 0, None, 1.0)])
    return dx


# ---------------------------------------------------------------- DenseConcat
def dense_fwd(W1, b1, W2, b2, midi, audio, drop_p=0.0, seed=0, seed_dev=None):
    """DenseConcat.forward (model.py:102-108): cat(audio, midi) -> fc1 -> ReLU -> Dropout
    -> fc2 -> ReLU -> Dropout, computed in NCL (no transposes)."""
    B, _, T = midi.shape
    h1 = _e((B, W1.shape[0], T), midi)
    K.linear_fwd([(audio, 0), (midi, 0)], W1, b1, h1, act=RELU, drop_p=drop_p, seed=seed,
                 seed_dev=seed_dev)
    h2 = _e((B, W2.shape[0], T), midi)
    K.linear_fwd([(h1, 0)], W2, b2, h2, act=RELU, drop_p=drop_p, seed=seed + 1, seed_dev=seed_dev)
    return h2, (midi, audio, h1, h2, drop_p)


def dense_bwd(params, saved, sink, d_h2, need_dx=True, gated=False):
    """gated=True: d_h2 already is d(fc2 pre-activation) (gate applied by the producer)."""
    W1, b1, W2, b2 = params
    midi, audio, h1, h2, drop_p = saved
    s = 1.0 / (1.0 - drop_p)
    dpre2 = d_h2 if gated else K.relu_gate_bwd(d_h2, h2, s)
    g, acc = sink.target(W2)
    sink.wgrad(lambda: K.linear_wgrad(dpre2, [(h1, 0)], g, acc), dpre2, h1)
    g, acc = sink.target(b2)
    K.bias_grad(dpre2, g, acc)
    dpre1 = torch.empty_like(h1)
    K.linear_dgrad(dpre2, W2, [(dpre1, 0, h1, s)])
    del dpre2
    g, acc = sink.target(W1)
    sink.wgrad(lambda: K.linear_wgrad(dpre1, [(audio, 0), (midi, 0)], g, acc), dpre1, audio, midi)
    g, acc = sink.target(b1)
    K.bias_grad(dpre1, g, acc)
    if not need_dx:
        return None, None
    d_audio = torch.empty_like(audio)
    d_midi = torch.empty_like(midi)
    K.linear_dgrad(dpre1, W1, [(d_audio, 0, None, 1.0), (d_midi, 0, None, 1.0)])
    return d_midi, d_audio


# --------------------------------------------------------------------- UpConv
def crop_offset(L_bypass, L_up):
    """crop_and_concat (model.py:71-77) == bypass shifted by c = (Lb - Lu)//2."""
    return (L_bypass - L_up) // 2


def upconv_fwd(Wu, bu, W1, b1, W2, b2, res, dec, cond):
    """UpConv.forward (model.py:80-90)."""
    B, _, Tin = dec.shape
    k = Wu.shape[2]
    Co = Wu.shape[1]
    Lu = K.convT2_out_len(Tin, k)
    u_pre = _e((B, Co, Lu), dec)
    K.convT2_fwd(dec, Wu, bu, u_pre)
    u, _, mu_, ru_ = K.in_lrelu_fwd(u_pre, False)
    c_res = crop_offset(res.shape[2], Lu)
    v_pre = _e((B, Co, Lu), dec)
    K.conv3_fwd([(u, 0), (res, c_res)], W1, b1, v_pre)
    v, _, mv_, rv_ = K.in_lrelu_fwd(v_pre, False)
    srcs2 = [(v, 0)]
    c_cond = 0
    if cond is not None:
        c_cond = crop_offset(cond.shape[2], Lu)
        srcs2.append((cond, c_cond))
    w_pre = _e((B, Co, Lu), dec)
    K.conv3_fwd(srcs2, W2, b2, w_pre)
    w, _, mw_, rw_ = K.in_lrelu_fwd(w_pre, False)
    saved = (dec, u_pre, mu_, ru_, u, res, c_res, v_pre, mv_, rv_, v, cond, c_cond, w_pre, mw_, rw_)
    return w, saved


def _grad_buffer_for_bypass(t, c, Lu):
    """Gradient buffer of a crop_and_concat bypass: positions s with s - c outside [0, Lu)
    never reach the output and must read zero (only when the crop trims the bypass)."""
    covered = c <= 0 and t.shape[2] - c <= Lu
    return torch.empty_like(t) if covered else torch.zeros_like(t)


def upconv_bwd(params, saved, sink, d_w, res_gate=None, res_gate_scale=1.0, dec_gate=None,
               dec_gate_scale=1.0):
    """Returns (d_res, d_dec, d_cond). res_gate/dec_gate apply a producer DenseConcat's
    ReLU/dropout backward inside the dgrad epilogues (the result is d(fc2 pre-activation))."""
    Wu, bu, W1, b1, W2, b2 = params
    (dec, u_pre, mu_, ru_, u, res, c_res, v_pre, mv_, rv_, v, cond, c_cond, w_pre, mw_,
     rw_) = saved
    dw_pre, rs_w = K.in_lrelu_bwd(w_pre, mw_, rw_, d_w, rowsum=True)
    srcs2 = [(v, 0)] + ([(cond, c_cond)] if cond is not None else [])
    g, acc = sink.target(W2)
    sink.wgrad(lambda: K.conv3_wgrad(dw_pre, srcs2, g, acc), dw_pre, *(t for t, _ in srcs2))
    g, acc = sink.target(b2)
    K.bias_grad_rows(rs_w, g, acc)
    dv = torch.empty_like(v)
    dsts = [(dv, 0, None, 1.0)]
    d_cond = None
    if cond is not None:
        d_cond = _grad_buffer_for_bypass(cond, c_cond, v.shape[2])
        dsts.append((d_cond, c_cond, None, 1.0))
    K.conv3_dgrad(dw_pre, W2, dsts)
    del dw_pre
    dv_pre, rs_v = K.in_lrelu_bwd(v_pre, mv_, rv_, dv, rowsum=True)
    del dv
    g, acc = sink.target(W1)
    sink.wgrad(lambda: K.conv3_wgrad(dv_pre, [(u, 0), (res, c_res)], g, acc), dv_pre, u, res)
    g, acc = sink.target(b1)
    K.bias_grad_rows(rs_v, g, acc)
    du = torch.empty_like(u)
    d_res = _grad_buffer_for_bypass(res, c_res, u.shape[2])
    K.conv3_dgrad(dv_pre, W1, [(du, 0, None, 1.0), (d_res, c_res, res_gate, res_gate_scale)])
    del dv_pre
    du_pre, rs_u = K.in_lrelu_bwd(u_pre, mu_, ru_, du, rowsum=True)
    del du
    g, acc = sink.target(Wu)
    sink.wgrad(lambda: K.convT2_wgrad(dec, du_pre, g, acc), dec, du_pre)
    g, acc = sink.target(bu)
    K.bias_grad_rows(rs_u, g, acc)
    d_dec = torch.empty_like(dec)
    K.convT2_dgrad(du_pre, Wu, [(d_dec, 0, dec_gate, dec_gate_scale)])
    return d_res, d_dec, d_cond


# ----------------------------------------------------------- whole network
MBR_SCALE = 16.0  # 4 MBRBlocks x (returns 2*x), model.py:172-173,295-298


def _pp(P, prefix, names):
    return tuple(P[f"{prefix}.{n}"] for n in names)


DC = ("conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias")
DN = ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias")
UP = ("upconv.weight", "upconv.bias", "conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias")


def _record(obj, stream):
    """record_stream(stream) on every tensor of a nested tuple / list: tensors made on one stream
    and used on another must not be handed out again by the caching allocator before the other
    stream's kernels are done with them."""
    if isinstance(obj, torch.Tensor):
        obj.record_stream(stream)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _record(o, stream)


def _encoder_fwd(P, name, x, depth, enc, svs):
    for i in range(depth):
        x, before, sv = downconv_fwd(*_pp(P, f"{name}.{i}", DC), x, i < depth - 1)
        enc.append(before)
        svs.append(sv)
    return x


def network_fwd(P, x_midi, x_audio, cond, drop_p=0.0, seed=0, depth=5, seed_dev=None, aux=None):
    """PerformanceNet.forward (model.py:262-300) as one kernel program. seed_dev (optional
    int64 device scalar) is added to every dropout seed on the device (hipGraph replays).

    aux (optional stream): the audio encoder runs on it, concurrently with the MIDI and
    onset/offset encoders on the current stream (independent branches until dense_concats.0;
    their deep levels are a few hundred workgroups each, so one alone leaves the chip idle).
    Same kernels, same results."""
    enc_m, enc_a, sv_m, sv_a = [], [], [], []
    main = torch.cuda.current_stream()
    if aux is not None:
        aux.wait_stream(main)
        x_audio.record_stream(aux)
    xm = _encoder_fwd(P, "down_convs", x_midi, depth, enc_m, sv_m)
    if aux is not None:
        with torch.cuda.stream(aux):
            xa = _encoder_fwd(P, "down_convs_audio", x_audio, depth, enc_a, sv_a)
    else:
        xa = _encoder_fwd(P, "down_convs_audio", x_audio, depth, enc_a, sv_a)
    conds, sv_o = [], []
    c = cond
    for i in range(3):
        c, _, sv = downconv_fwd(*_pp(P, f"onset_offset_encoder.down_convs.{i}", DC), c, True)
        sv_o.append(sv)
        if i > 0:
            conds.append(c)
    skips, sv_dn, ev = [None] * 4, [None] * 4, [None] * 4
    if aux is not None:
        main.wait_stream(aux)  # the audio encoder (recorded before the dense levels are queued)
        _record((xa, enc_a, sv_a), main)
        # the skip levels' DenseConcats need only the encoders: they run on aux beside
        # dense_concats.0 and the up-convolution chain, which waits for each level's event
        aux.wait_stream(main)
        _record(enc_m, aux)
        with torch.cuda.stream(aux):
            for i in range(4):
                skips[i], sv_dn[i] = dense_fwd(*_pp(P, f"dense_concats.{i + 1}", DN), enc_m[-(i + 2)],
                                               enc_a[-(i + 2)], drop_p, seed + 2 * (i + 1), seed_dev)
                ev[i] = torch.cuda.Event()
                ev[i].record(aux)
        _record((skips, sv_dn), main)
    x, sv_d0 = dense_fwd(*_pp(P, "dense_concats.0", DN), xm, xa, drop_p, seed, seed_dev)
    sv_up = []
    for i in range(4):
        if aux is None:
            skips[i], sv_dn[i] = dense_fwd(*_pp(P, f"dense_concats.{i + 1}", DN), enc_m[-(i + 2)],
                                           enc_a[-(i + 2)], drop_p, seed + 2 * (i + 1), seed_dev)
        else:
            main.wait_event(ev[i])
        cd = conds[i - 1] if i < 2 else None
        x, svu = upconv_fwd(*_pp(P, f"up_convs.{i}", UP), skips[i], x, cd)
        sv_up.append(svu)
    W, b = P["lastconv.weight"], P["lastconv.bias"]
    B, _, T = x.shape
    y = _e((B, W.shape[1], T), x)
    K.convT1_fwd(x, W, b, y, alpha=MBR_SCALE, act=LRELU)
    state = dict(sv_m=sv_m, sv_a=sv_a, sv_d0=sv_d0, sv_o=sv_o, sv_dn=sv_dn, sv_up=sv_up, x_dec=x,
                 y=y, depth=depth)
    return y, state


def backward_param_order(depth=5):
    """Parameter names in the order network_bwd produces their gradients (the flat buffer's
    layout, so data-parallel buckets complete front to back during the backward pass)."""
    names = ["lastconv.weight", "lastconv.bias"]
    blk = lambda prefix, group: [f"{prefix}.{n}" for n in group]  # noqa: E731
    for i in reversed(range(depth - 1)):
        names += blk(f"up_convs.{i}", UP[4:] + UP[2:4] + UP[:2])
        names += blk(f"dense_concats.{i + 1}", DN[2:] + DN[:2])
    names += blk("dense_concats.0", DN[2:] + DN[:2])
    for i in (2, 1, 0):
        names += blk(f"onset_offset_encoder.down_convs.{i}", DC[2:] + DC[:2])
    for name in ("down_convs", "down_convs_audio"):
        for i in reversed(range(depth)):
            names += blk(f"{name}.{i}", DC[2:] + DC[:2])
    return names


def network_bwd(P, st, dy, sink, need_input_grads=(False, False, False), aux=None):
    main = torch.cuda.current_stream()
    depth = st["depth"]
    y = st["y"]
    dypre = K.lrelu_bwd(dy, y)
    W = P["lastconv.weight"]
    x_dec = st["x_dec"]
    g, acc = sink.target(W)
    sink.wgrad(lambda: K.convT1_wgrad(x_dec, dypre, g, acc, scale=MBR_SCALE), x_dec, dypre)
    g, acc = sink.target(P["lastconv.bias"])
    K.bias_grad(dypre, g, acc)
    dx = torch.empty_like(x_dec)
    K.convT1_dgrad(dypre, W, dx, alpha=MBR_SCALE)
    # a block is done once its weights are read for the last time (its dgrad): listeners may
    # then update them (train.BackwardAdam), not just reduce their gradients
    sink.block_done()
    del dypre
    d_before_m = [None] * depth
    d_before_a = [None] * depth
    d_conds = [None, None]
    sv_d0 = st["sv_d0"]
    for i in reversed(range(4)):
        svd = st["sv_dn"][i]
        s = 1.0 / (1.0 - svd[4])
        dec_gate = sv_d0[3] if i == 0 else None  # up_convs[0]'s input is dense_concats[0]'s output
        d_res_pre, dx, d_cd = upconv_bwd(_pp(P, f"up_convs.{i}", UP), st["sv_up"][i], sink, dx,
                                         res_gate=svd[3], res_gate_scale=s, dec_gate=dec_gate,
                                         dec_gate_scale=1.0 / (1.0 - sv_d0[4]))
        sink.block_done()
        if i < 2:
            d_conds[(i - 1) % 2] = d_cd
        if aux is not None:
            # the skip level's DenseConcat backward feeds only the encoders' backward: on aux,
            # beside the up-convolution chain
            aux.wait_stream(main)
            _record((d_res_pre, svd), aux)
            with torch.cuda.stream(aux):
                d_midi, d_audio = dense_bwd(_pp(P, f"dense_concats.{i + 1}", DN), svd, sink,
                                            d_res_pre, gated=True)
                sink.block_done()
            d_midi.record_stream(main)
        else:
            d_midi, d_audio = dense_bwd(_pp(P, f"dense_concats.{i + 1}", DN), svd, sink, d_res_pre,
                                        gated=True)
            sink.block_done()
        d_before_m[depth - 2 - i] = d_midi
        d_before_a[depth - 2 - i] = d_audio
    d_xm, d_xa = dense_bwd(_pp(P, "dense_concats.0", DN), sv_d0, sink, dx, gated=True)
    sink.block_done()
    del dx
    # onset/offset encoder: level 2 pooled = conds[1], level 1 pooled = conds[0] and level-2 input
    sv_o = st["sv_o"]
    d2 = downconv_bwd(_pp(P, "onset_offset_encoder.down_convs.2", DC), sv_o[2], sink,
                      d_pool0=d_conds[1])
    sink.block_done()
    d1 = downconv_bwd(_pp(P, "onset_offset_encoder.down_convs.1", DC), sv_o[1], sink,
                      d_pool0=d_conds[0], d_pool1=d2)
    sink.block_done()
    del d2
    d_cond_in = downconv_bwd(_pp(P, "onset_offset_encoder.down_convs.0", DC), sv_o[0], sink,
                             d_pool0=d1, need_dx=need_input_grads[2])
    sink.block_done()
    del d1
    def encoder_bwd(name, sv, d_before, d_top):
        d_pool = None
        for i in reversed(range(depth)):
            prm = _pp(P, f"{name}.{i}", DC)
            if i == depth - 1:  # no pooling: before_pool is the output
                d_pool = downconv_bwd(prm, sv[i], sink, d_before=d_top, need_dx=True)
                sink.block_done()
            else:
                need = i > 0 or need_input_grads[0 if name == "down_convs" else 1]
                d_pool = downconv_bwd(prm, sv[i], sink, d_before=d_before[i], d_pool0=d_pool,
                                      need_dx=need)
            sink.block_done()
            d_before[i] = None
        return d_pool

    # the two encoders' backward are independent: with an aux stream the audio encoder's runs on
    # it beside the MIDI encoder's (enqueued second, so blocks finish in the flat-buffer order)
    if aux is not None:
        main.wait_stream(aux)  # the skip levels' DenseConcat backward (d_before_m)
    g_m = encoder_bwd("down_convs", st["sv_m"], d_before_m, d_xm)
    if aux is not None:
        aux.wait_stream(main)
        _record((d_before_a, d_xa, st["sv_a"]), aux)
        with torch.cuda.stream(aux):
            g_a = encoder_bwd("down_convs_audio", st["sv_a"], d_before_a, d_xa)
        main.wait_stream(aux)
        if g_a is not None:
            g_a.record_stream(main)
    else:
        g_a = encoder_bwd("down_convs_audio", st["sv_a"], d_before_a, d_xa)
    sink.join()
    return g_m, g_a, d_cond_in


class PerformanceNetFunction(torch.autograd.Function):
    """One autograd node for the whole network. Inputs: (module, x_midi, x_audio, cond, *params)."""

    @staticmethod
    def forward(ctx, module, x_midi, x_audio, cond, *params):
        P = module._param_dict()
        drop_p = module._dropout_p() if module.training else 0.0
        seed = module._next_seed() if drop_p > 0 else 0
        xm, xa, cd = (t if t.stride(2) == 1 and t.dtype == torch.float32 else t.float().contiguous()
                      for t in (x_midi, x_audio, cond))
        y, state = network_fwd(P, xm, xa, cd, drop_p, seed, module.depth,
                               module.__dict__.get("_mst_seed_dev") if drop_p > 0 else None,
                               aux=module._enc_stream())
        ctx.module = module
        ctx.state = state
        return y

    @staticmethod
    def backward(ctx, dy):
        module = ctx.module
        P = module._param_dict()
        need = (ctx.needs_input_grad[1], ctx.needs_input_grad[2], ctx.needs_input_grad[3])
        # block-completion listeners, in order: dp.OverlappedAllReduce (bucket all-reduces), then
        # train.BackwardAdam (bucket updates, after their all-reduce)
        hooks = [h for h in (getattr(module, "_mst_dp", None), getattr(module, "_mst_adam", None))
                 if h is not None]
        for h in hooks:
            h.begin()

        def on_ready(params):
            for h in hooks:
                h.ready(params)
        sink = module._grad_sink(on_ready if hooks else None)
        g_m, g_a, g_c = network_bwd(P, ctx.state, dy.contiguous(), sink, need,
                                    aux=module._enc_stream())
        # the side stream's join event (None when the weight gradients ran on the compute
        # stream): an Event, so no hook closure of this backward outlives it
        module.__dict__["_mst_wgrad_joined"] = sink.joined
        module.__dict__["_mst_bwd_blocks"] = sink.block
        for h in hooks:
            h.launch_remaining()
        ctx.state = None
        n_params = len(module._flat_params_list())
        return (None, g_m if need[0] else None, g_a if need[1] else None,
                g_c if need[2] else None) + (None,) * n_params


def l1_loss(pred, target):
    """nn.L1Loss() (train.py:132): mean |pred - target| on the device (torch.ops.mst.l1_loss;
    its registered backward is mst::l1_loss_backward)."""
    return torch.ops.mst.l1_loss(pred, target)


def mse_loss(pred, target):
    """nn.MSELoss() forward (test(), train.py:158); evaluation only (torch.ops.mst.mse_loss)."""
    return torch.ops.mst.mse_loss(pred, target)
