# coding: utf-8
"""The C ABI (``include/abcd_hip.h``) registered as PyTorch custom operators
(``torch.library``, namespace ``abcd``) with their autograd formulas -- the
operator boundary the module classes of ``model.py`` call.

One operator per reference method on the hot path, and one per backward:

=========================  ==============================================  =========================================
operator                   replaces (reference)                            C entry point
=========================  ==============================================  =========================================
``abcd::encoder``          ``RNN_Variational_Encoder.forward`` model.py:60  ``abcd_encoder_forward_dropout``
``abcd::encoder_bwd``      its autograd backward                           ``abcd_encoder_backward_dropout``
``abcd::sampler``          ``ABCDSampler.forward`` model.py:581 /           ``abcd_sampler_forward``
                           ``Sampler.forward`` plain/model.py:552
``abcd::sampler_bwd``      its backward                                    ``abcd_sampler_forward_backward``
``abcd::sampler_sample``   ``ABCDSampler.sample`` model.py:592             ``abcd_sampler_sample``
``abcd::sampler_sample_bwd``                                               ``abcd_sampler_sample_backward``
``abcd::sampler_kl``       ``ABCDSampler.kl_divergence`` model.py:608      ``abcd_sampler_kl``
``abcd::sampler_kl_bwd``                                                   ``abcd_sampler_kl_backward``
``abcd::decoder``          ``RNN_Variational_Decoder.forward`` model.py:147 ``abcd_decoder_forward_dropout``
``abcd::decoder_bwd``      its backward (emission + offset losses)         ``abcd_decoder_backward_dropout``
``abcd::linear``           ``MLP`` layers (Linear [+ Tanh]) model.py:316   ``abcd_linear``
``abcd::linear_bwd``       their backward                                  ``abcd_linear_backward``
=========================  ==============================================  =========================================

Operators take tensors, ints and floats only (no module objects): the
configuration travels as an ``int[]`` in the C struct's field order, the
parameters as a ``Tensor[]`` in the module's parameter order.  The forward
operators also return the kernels' workspace (a uint8 tensor holding the
forward stash the backward reads), so every operator is functional (autograd
formulas need that): ``sampler_sample`` and ``sampler_kl`` each stash into a
workspace of their own.  Philox keys (64-bit) cross the schema as
two's-complement int64.

Every operator runs the HIP kernels on the tensors' device; there is no CPU
kernel (a CPU tensor raises, as everywhere on the product path)."""
from typing import List, Optional, Sequence

import torch

from . import _native as N

Tensor = torch.Tensor
_U64 = (1 << 64) - 1


def _i64(x):
    """uint64 -> int64 (two's complement) for the schema."""
    x = int(x) & _U64
    return x - (1 << 64) if x >= (1 << 63) else x


def _u64(x):
    return int(x) & _U64


def _packed(data, batch_sizes, F, L=None):
    bs = batch_sizes
    if bs.dtype != torch.int64 or bs.device.type != "cpu":
        bs = bs.to("cpu", torch.int64)
    bs = bs.contiguous()
    st = N.Packed()
    st.data = data.data_ptr() if data is not None else None
    st.batch_sizes = bs.data_ptr()
    st.T = int(bs.numel())
    st.L = int(data.shape[0]) if data is not None else int(bs.sum()) if L is None else int(L)
    st.B = int(bs[0])
    st.F = int(F)
    return st, bs


def _ptrs(ts):
    return [None if t is None else t.data_ptr() for t in ts]


# ----------------------------------------------------------------------------
# encoder
# ----------------------------------------------------------------------------
def _enc_cfg(cfg):
    c = N.EncoderCfg()
    c.input_size, c.hidden_size, c.rnn_type, c.layers, c.bidirectional = (int(v) for v in cfg)
    return c


def _enc_struct(cfg, ts):
    """ts: (w_ih, w_hh, b_ih, b_hh) per (layer, direction), layer-major."""
    st = N.EncoderParams()
    dirs = 2 if cfg[4] else 1
    for i in range(int(cfg[3]) * dirs):
        l, d = divmod(i, dirs)
        st.w[l][d].w_ih, st.w[l][d].w_hh, st.w[l][d].b_ih, st.w[l][d].b_hh = _ptrs(ts[4 * i:4 * i + 4])
    return st


def _enc_out_width(cfg):
    w = int(cfg[3]) * int(cfg[1]) * (2 if cfg[4] else 1)
    return w * 2 if int(cfg[2]) == N.LSTM else w


@torch.library.custom_op("abcd::encoder", mutates_args=())
def encoder(data: Tensor, batch_sizes: Tensor, weights: List[Tensor], noise: List[Tensor],
            cfg: List[int]) -> List[Tensor]:
    """-> [last hidden (B x hidden_size_total), workspace].  noise: the
    inter-layer dropout masks (layers - 1 of them) or [] (no dropout)."""
    N.require_gpu(data)
    L = N.lib()
    c = _enc_cfg(cfg)
    pk, bs = _packed(data, batch_sizes, cfg[0])
    nbytes = L.abcd_encoder_workspace_bytes(c, pk.T, pk.L, pk.B)
    if nbytes == 0:
        raise N.HipError("encoder: unsupported configuration (hidden size must be a multiple of 16)")
    ws = N.workspace(nbytes, data.device)
    out = torch.empty(pk.B, _enc_out_width(cfg), device=data.device)
    N.check(L.abcd_encoder_forward_dropout(c, _enc_struct(cfg, weights), pk, N.ptr_array(list(noise) or None), N.ptr(out),
                                           N.ptr(ws), ws.numel(), N.stream()), "encoder forward")
    N.op_status.probe(data.device, "encoder forward")
    return [out, ws]


@encoder.register_fake
def _(data, batch_sizes, weights, noise, cfg):
    B = batch_sizes[0] if batch_sizes.numel() else 0
    return [data.new_empty(int(B), _enc_out_width(cfg)), data.new_empty(0, dtype=torch.uint8)]


@torch.library.custom_op("abcd::encoder_bwd", mutates_args=())
def encoder_bwd(data: Tensor, batch_sizes: Tensor, weights: List[Tensor], noise: List[Tensor],
                ws: Tensor, d_out: Tensor, cfg: List[int]) -> List[Tensor]:
    c = _enc_cfg(cfg)
    pk, bs = _packed(data, batch_sizes, cfg[0])
    grads = [torch.empty_like(w) for w in weights]
    N.check(N.lib().abcd_encoder_backward_dropout(c, _enc_struct(cfg, weights), pk, N.ptr_array(list(noise) or None),
                                                  N.ptr(d_out.contiguous()), _enc_struct(cfg, grads), N.ptr(ws),
                                                  ws.numel(), N.stream(), None), "encoder backward")
    N.op_status.probe(data.device, "encoder backward")
    return grads


@encoder_bwd.register_fake
def _(data, batch_sizes, weights, noise, ws, d_out, cfg):
    return [torch.empty_like(w) for w in weights]


def _encoder_setup(ctx, inputs, output):
    data, batch_sizes, weights, noise, cfg = inputs
    ctx.data, ctx.batch_sizes, ctx.weights, ctx.noise, ctx.cfg = data, batch_sizes, weights, noise, cfg
    ctx.ws = output[1]
    ctx.mark_non_differentiable(output[1])


def _encoder_backward(ctx, grads):
    d_out = grads[0]
    g = encoder_bwd(ctx.data, ctx.batch_sizes, list(ctx.weights), ctx.noise, ctx.ws, d_out, list(ctx.cfg))
    return None, None, g, [None] * len(ctx.noise), None


encoder.register_autograd(_encoder_backward, setup_context=_encoder_setup)


# ----------------------------------------------------------------------------
# samplers (ABCD: cfg[4] == 0; plain Gaussian: cfg[4] == 1)
# ----------------------------------------------------------------------------
def _samp_cfg(cfg):
    """cfg: [input_size, mlp_hidden, num_categories, feature_dim, plain(, valid_categories, valid_feature_dim)]"""
    c = N.SamplerCfg()
    v = [int(x) for x in cfg] + [0] * (7 - len(cfg))
    (c.input_size, c.mlp_hidden, c.num_categories, c.feature_dim, c.plain, c.valid_categories,
     c.valid_feature_dim) = v
    return c


def _samp_struct(cfg, mlp, codebook=None, psl=None, prior=1.0):
    st = N.SamplerParams()
    for k in range(len(mlp) // 4):
        st.mlp[k].w1, st.mlp[k].b1, st.mlp[k].w2, st.mlp[k].b2 = _ptrs(mlp[4 * k:4 * k + 4])
    st.codebook = None if codebook is None else codebook.data_ptr()
    st.posterior_shape_logits = None if psl is None else psl.data_ptr()
    st.prior_concentration = float(prior)
    return st


def _logit_width(cfg):
    return 2 * int(cfg[3]) if cfg[4] else int(cfg[2])


def _sampler_ws(cfg, B, device):
    nbytes = N.lib().abcd_sampler_workspace_bytes(_samp_cfg(cfg), B)
    if nbytes == 0:
        raise N.HipError("sampler: unsupported configuration (sizes must be multiples of 16)")
    return N.workspace(nbytes, device)


@torch.library.custom_op("abcd::sampler", mutates_args=())
def sampler(h: Tensor, mlp: List[Tensor], codebook: Optional[Tensor], cfg: List[int]) -> List[Tensor]:
    """-> [logits (B x K; plain: [mean | log_var], B x 2f), workspace]"""
    N.require_gpu(h)
    h = h.contiguous()
    B = h.shape[0]
    ws = _sampler_ws(cfg, B, h.device)
    out = torch.empty(B, _logit_width(cfg), device=h.device)
    N.check(N.lib().abcd_sampler_forward(_samp_cfg(cfg), _samp_struct(cfg, mlp, codebook), N.ptr(h), B, N.ptr(out),
                                         N.ptr(ws), ws.numel(), N.stream()), "sampler forward")
    return [out, ws]


@sampler.register_fake
def _(h, mlp, codebook, cfg):
    return [h.new_empty(h.shape[0], _logit_width(cfg)), h.new_empty(0, dtype=torch.uint8)]


@torch.library.custom_op("abcd::sampler_bwd", mutates_args=())
def sampler_bwd(h: Tensor, mlp: List[Tensor], codebook: Optional[Tensor], ws: Tensor, d_logits: Tensor,
                cfg: List[int]) -> List[Tensor]:
    """-> [d_h, d_mlp..., (d_codebook)]"""
    h = h.contiguous()
    d_h = torch.empty_like(h)
    gm = [torch.empty_like(t) for t in mlp]
    gc = None if codebook is None else torch.empty_like(codebook)
    g = N.SamplerGrads()
    for k in range(len(mlp) // 4):
        g.mlp[k].w1, g.mlp[k].b1, g.mlp[k].w2, g.mlp[k].b2 = _ptrs(gm[4 * k:4 * k + 4])
    g.codebook = None if gc is None else gc.data_ptr()
    N.check(N.lib().abcd_sampler_forward_backward(_samp_cfg(cfg), _samp_struct(cfg, mlp, codebook), N.ptr(h),
                                                  h.shape[0], N.ptr(d_logits.contiguous()), N.ptr(d_h), g, 0,
                                                  N.ptr(ws), ws.numel(), N.stream()), "sampler forward backward")
    return [d_h] + gm + ([] if gc is None else [gc])


@sampler_bwd.register_fake
def _(h, mlp, codebook, ws, d_logits, cfg):
    return [torch.empty_like(h)] + [torch.empty_like(t) for t in mlp] + ([] if codebook is None
                                                                         else [torch.empty_like(codebook)])


def _sampler_setup(ctx, inputs, output):
    h, mlp, codebook, cfg = inputs
    ctx.h, ctx.mlp, ctx.codebook, ctx.cfg, ctx.ws = h, mlp, codebook, cfg, output[1]
    ctx.mark_non_differentiable(output[1])


def _sampler_backward(ctx, grads):
    g = sampler_bwd(ctx.h, list(ctx.mlp), ctx.codebook, ctx.ws, grads[0], list(ctx.cfg))
    nm = len(ctx.mlp)
    return g[0], g[1:1 + nm], (g[1 + nm] if ctx.codebook is not None else None), None


sampler.register_autograd(_sampler_backward, setup_context=_sampler_setup)


@torch.library.custom_op("abcd::sampler_sample", mutates_args=())
def sampler_sample(logits: Tensor, codebook: Optional[Tensor], cfg: List[int], mode: int, temperature: float,
                   noise: Optional[Tensor], seed: int, offset: int) -> List[Tensor]:
    """-> [feats (B x D), workspace]: ABCD Gumbel-softmax / softmax y C^T;
    plain mu + e^{lv/2} eps.  The workspace holds the stash its backward reads."""
    N.require_gpu(logits)
    logits = logits.contiguous()
    B = logits.shape[0]
    ws = _sampler_ws(cfg, B, logits.device)
    feats = torch.empty(B, int(cfg[3]), device=logits.device)
    N.check(N.lib().abcd_sampler_sample(_samp_cfg(cfg), _samp_struct(cfg, [], codebook), N.ptr(logits), B,
                                        int(mode), float(temperature), N.ptr(noise), _u64(seed), _u64(offset),
                                        N.ptr(feats), N.ptr(ws), ws.numel(), N.stream()), "sampler sample")
    return [feats, ws]


@sampler_sample.register_fake
def _(logits, codebook, cfg, mode, temperature, noise, seed, offset):
    return [logits.new_empty(logits.shape[0], int(cfg[3])), logits.new_empty(0, dtype=torch.uint8)]


@torch.library.custom_op("abcd::sampler_sample_bwd", mutates_args=())
def sampler_sample_bwd(ws: Tensor, codebook: Optional[Tensor], d_feats: Tensor, cfg: List[int], B: int, mode: int,
                       temperature: float) -> List[Tensor]:
    """-> [d_logits, (d_codebook)]"""
    d_logits = torch.empty(B, _logit_width(cfg), device=d_feats.device)
    d_cb = None if codebook is None else torch.empty_like(codebook)
    N.check(N.lib().abcd_sampler_sample_backward(_samp_cfg(cfg), _samp_struct(cfg, [], codebook), B, int(mode),
                                                 float(temperature), N.ptr(d_feats.contiguous()), N.ptr(d_logits),
                                                 N.ptr(d_cb), N.ptr(ws), ws.numel(), N.stream()),
            "sampler sample backward")
    return [d_logits] + ([] if d_cb is None else [d_cb])


@sampler_sample_bwd.register_fake
def _(ws, codebook, d_feats, cfg, B, mode, temperature):
    return [d_feats.new_empty(B, _logit_width(cfg))] + ([] if codebook is None else [torch.empty_like(codebook)])


def _sample_setup(ctx, inputs, output):
    logits, codebook, cfg, mode, temperature, noise, seed, offset = inputs
    ctx.ws, ctx.codebook, ctx.cfg, ctx.mode, ctx.tau, ctx.B = output[1], codebook, cfg, mode, temperature, \
        logits.shape[0]
    ctx.mark_non_differentiable(output[1])


def _sample_backward(ctx, grads):
    g = sampler_sample_bwd(ctx.ws, ctx.codebook, grads[0], list(ctx.cfg), ctx.B, ctx.mode, ctx.tau)
    return g[0], (g[1] if ctx.codebook is not None else None), None, None, None, None, None, None


sampler_sample.register_autograd(_sample_backward, setup_context=_sample_setup)


@torch.library.custom_op("abcd::sampler_kl", mutates_args=())
def sampler_kl(logits: Tensor, psl: Optional[Tensor], cfg: List[int], prior: float,
               entire_data_size: float) -> List[Tensor]:
    """-> [KL scalar, workspace]: ABCD Dirichlet-categorical; plain Gaussian"""
    N.require_gpu(logits)
    logits = logits.contiguous()
    ws = _sampler_ws(cfg, logits.shape[0], logits.device)
    kl = torch.empty((), device=logits.device)
    N.check(N.lib().abcd_sampler_kl(_samp_cfg(cfg), _samp_struct(cfg, [], None, psl, prior), N.ptr(logits),
                                    logits.shape[0], float(entire_data_size), N.ptr(kl), N.ptr(ws), ws.numel(),
                                    N.stream()), "sampler kl")
    return [kl, ws]


@sampler_kl.register_fake
def _(logits, psl, cfg, prior, entire_data_size):
    return [logits.new_empty(()), logits.new_empty(0, dtype=torch.uint8)]


@torch.library.custom_op("abcd::sampler_kl_bwd", mutates_args=())
def sampler_kl_bwd(ws: Tensor, psl: Optional[Tensor], d_kl: Tensor, cfg: List[int], B: int, prior: float,
                   entire_data_size: float) -> List[Tensor]:
    """-> [d_logits, (d_posterior_shape_logits)]"""
    d_logits = torch.empty(B, _logit_width(cfg), device=d_kl.device)
    d_psl = None if psl is None else torch.empty_like(psl)
    N.check(N.lib().abcd_sampler_kl_backward(_samp_cfg(cfg), _samp_struct(cfg, [], None, psl, prior), B,
                                             float(entire_data_size), N.ptr(d_kl.reshape(()).contiguous()), 0,
                                             N.ptr(d_logits), N.ptr(d_psl), N.ptr(ws), ws.numel(), N.stream()),
            "sampler kl backward")
    return [d_logits] + ([] if d_psl is None else [d_psl])


@sampler_kl_bwd.register_fake
def _(ws, psl, d_kl, cfg, B, prior, entire_data_size):
    return [d_kl.new_empty(B, _logit_width(cfg))] + ([] if psl is None else [torch.empty_like(psl)])


def _kl_setup(ctx, inputs, output):
    logits, psl, cfg, prior, n = inputs
    ctx.ws, ctx.psl, ctx.cfg, ctx.prior, ctx.n, ctx.B = output[1], psl, cfg, prior, n, logits.shape[0]
    ctx.mark_non_differentiable(output[1])


def _kl_backward(ctx, grads):
    g = sampler_kl_bwd(ctx.ws, ctx.psl, grads[0], list(ctx.cfg), ctx.B, ctx.prior, ctx.n)
    return g[0], (g[1] if ctx.psl is not None else None), None, None, None


sampler_kl.register_autograd(_kl_backward, setup_context=_kl_setup)


# ----------------------------------------------------------------------------
# decoder
# ----------------------------------------------------------------------------
def _dec_cfg(cfg):
    c = N.DecoderCfg()
    (c.output_size, c.hidden_size, c.mlp_hidden, c.feature_size, c.rnn_type, c.feedback, c.num_speakers,
     c.speaker_dim) = (int(v) for v in cfg)
    return c


def _dec_struct(cfg, ts):
    """ts: [embed_speaker (if cfg[6])] f2h_w f2h_b offset(4) mu(4) lv(4) cell(w_ih w_hh b_ih b_hh)"""
    st = N.DecoderParams()
    i = 0
    if int(cfg[6]):
        st.embed_speaker = None if ts[0] is None else ts[0].data_ptr()
        i = 1
    p = _ptrs(ts[i:])
    st.f2h_w, st.f2h_b = p[0], p[1]
    for name, k in (("offset", 2), ("mu", 6), ("lv", 10)):
        m = getattr(st, name)
        m.w1, m.b1, m.w2, m.b2 = p[k:k + 4]
    st.cell.w_ih, st.cell.w_hh, st.cell.b_ih, st.cell.b_hh = p[14:18]
    return st


@torch.library.custom_op("abcd::decoder", mutates_args=())
def decoder(features: Tensor, batch_sizes: Tensor, speaker: Optional[Tensor], gt: Optional[Tensor],
            gt_off: Optional[Tensor], eps: Optional[Tensor], seed: int, offset: int, xmask: Optional[Tensor],
            params: List[Tensor], cfg: List[int]) -> List[Tensor]:
    """-> [em, off, flat, mu, lv, offset_logits, workspace]; em / off are 0-d
    (0 when the target is absent); flat / mu / lv are L x F."""
    N.require_gpu(features)
    features = features.contiguous()
    L_ = N.lib()
    c = _dec_cfg(cfg)
    F = int(cfg[0])
    pk, bs = _packed(gt, batch_sizes, F)
    nbytes = L_.abcd_decoder_workspace_bytes(c, pk.T, pk.L, pk.B)
    if nbytes == 0:
        raise N.HipError("decoder: unsupported configuration (sizes must be multiples of 16)")
    dev = features.device
    ws = N.workspace(nbytes, dev)
    spk = speaker.to(dev, torch.int64).contiguous() if int(cfg[6]) else None
    flat = torch.empty(pk.L, F, device=dev)
    mu = torch.empty(pk.L, F, device=dev)
    lv = torch.empty(pk.L, F, device=dev)
    offl = torch.empty(pk.L, device=dev)
    losses = torch.zeros(2, device=dev)
    N.check(L_.abcd_decoder_forward_dropout(c, _dec_struct(cfg, params), pk, N.ptr(features), N.ptr(spk),
                                            N.ptr(None if gt_off is None else gt_off.contiguous()), N.ptr(eps),
                                            N.ptr(xmask), _u64(seed), _u64(offset), N.ptr(flat), N.ptr(mu),
                                            N.ptr(lv), N.ptr(offl), N.ptr(losses), N.ptr(ws), ws.numel(),
                                            N.stream()), "decoder forward")
    N.op_status.probe(dev, "decoder forward")
    return [losses[0].clone(), losses[1].clone(), flat, mu, lv, offl, ws]


@decoder.register_fake
def _(features, batch_sizes, speaker, gt, gt_off, eps, seed, offset, xmask, params, cfg):
    L = int(batch_sizes.sum())
    F = int(cfg[0])
    e = features.new_empty
    return [e(()), e(()), e(L, F), e(L, F), e(L, F), e(L), features.new_empty(0, dtype=torch.uint8)]


@torch.library.custom_op("abcd::decoder_bwd", mutates_args=())
def decoder_bwd(features: Tensor, batch_sizes: Tensor, speaker: Optional[Tensor], gt: Tensor, gt_off: Tensor,
                xmask: Optional[Tensor], params: List[Tensor], ws: Tensor, d_em: Tensor, d_off: Tensor,
                cfg: List[int]) -> List[Tensor]:
    """-> [d_features, d_params...]"""
    c = _dec_cfg(cfg)
    pk, bs = _packed(gt, batch_sizes, int(cfg[0]))
    dev = features.device
    spk = speaker.to(dev, torch.int64).contiguous() if int(cfg[6]) else None
    grads = [torch.empty_like(p) for p in params]
    d_features = torch.empty_like(features)
    N.check(N.lib().abcd_decoder_backward_dropout(c, _dec_struct(cfg, params), pk, N.ptr(features.contiguous()),
                                                  N.ptr(spk), N.ptr(gt_off.contiguous()), N.ptr(xmask),
                                                  N.ptr(d_em.reshape(()).contiguous()),
                                                  N.ptr(d_off.reshape(()).contiguous()), N.ptr(d_features),
                                                  _dec_struct(cfg, grads), N.ptr(ws), ws.numel(), N.stream(), None),
            "decoder backward")
    N.op_status.probe(dev, "decoder backward")
    return [d_features] + grads


@decoder_bwd.register_fake
def _(features, batch_sizes, speaker, gt, gt_off, xmask, params, ws, d_em, d_off, cfg):
    return [torch.empty_like(features)] + [torch.empty_like(p) for p in params]


def _decoder_setup(ctx, inputs, output):
    features, batch_sizes, speaker, gt, gt_off, eps, seed, offset, xmask, params, cfg = inputs
    ctx.saved = (features, batch_sizes, speaker, gt, gt_off, xmask, params, cfg)
    ctx.ws = output[6]
    ctx.mark_non_differentiable(*output[2:])  # per-frame outputs and the workspace: inspection only
    ctx.set_materialize_grads(False)


def _decoder_backward(ctx, grads):
    d_em, d_off = grads[0], grads[1]
    features, batch_sizes, speaker, gt, gt_off, xmask, params, cfg = ctx.saved
    if gt is None or gt_off is None:
        raise NotImplementedError("decoder backward needs ground_truth_out and ground_truth_offset "
                                  "(the losses it differentiates)")
    z = torch.zeros((), device=features.device)
    d_em = z if d_em is None else d_em
    d_off = z if d_off is None else d_off
    g = decoder_bwd(features, batch_sizes, speaker, gt, gt_off, xmask, list(params), ctx.ws, d_em, d_off, list(cfg))
    return g[0], None, None, None, None, None, None, None, None, g[1:], None


decoder.register_autograd(_decoder_backward, setup_context=_decoder_setup)


# ----------------------------------------------------------------------------
# nn.Linear (+ Tanh): the standalone MLP (model.py:316-334) outside the step
# ----------------------------------------------------------------------------
def _linear_ws(rows, cols, depth, device, backward=False):
    if backward:
        return N.workspace(N.lib().abcd_linear_backward_workspace_bytes(rows, cols, depth), device)
    Kp = (max(depth, cols) + 15) // 16 * 16
    return N.workspace((rows + cols) * Kp * 4 + (1 << 22), device)


@torch.library.custom_op("abcd::linear", mutates_args=())
def linear(x: Tensor, weight: Tensor, bias: Optional[Tensor], act: int) -> Tensor:
    """y = act(x W^T + b), act 0 = identity, 1 = tanh; x M x K, W N x K."""
    N.require_gpu(x)
    x = x.contiguous()
    weight = weight.contiguous()
    M, K = x.shape
    Nn = weight.shape[0]
    y = torch.empty(M, Nn, device=x.device)
    ws = _linear_ws(M, Nn, K, x.device)
    N.check(N.lib().abcd_linear(M, Nn, K, N.ptr(x), K, N.ptr(weight), K, N.ptr(None if bias is None else bias.contiguous()),
                                int(act), N.ptr(y), Nn, N.ptr(ws), ws.numel(), N.stream()), "linear")
    return y


@linear.register_fake
def _(x, weight, bias, act):
    return x.new_empty(x.shape[0], weight.shape[0])


@torch.library.custom_op("abcd::linear_bwd", mutates_args=())
def linear_bwd(x: Tensor, weight: Tensor, y: Tensor, dy: Tensor, act: int, need_bias: bool) -> List[Tensor]:
    """-> [dx, dW, db (empty when need_bias is false)]"""
    x, weight, y, dy = x.contiguous(), weight.contiguous(), y.contiguous(), dy.contiguous()
    M, K = x.shape
    Nn = weight.shape[0]
    dx = torch.empty_like(x)
    dW = torch.empty_like(weight)
    db = torch.empty(Nn if need_bias else 0, device=x.device)
    ws = _linear_ws(M, Nn, K, x.device, backward=True)
    N.check(N.lib().abcd_linear_backward(M, Nn, K, N.ptr(x), K, N.ptr(weight), K, N.ptr(y), Nn, int(act), N.ptr(dy),
                                         Nn, N.ptr(dx), K, N.ptr(dW), N.ptr(db) if need_bias else None, N.ptr(ws),
                                         ws.numel(), N.stream()), "linear backward")
    return [dx, dW, db]


@linear_bwd.register_fake
def _(x, weight, y, dy, act, need_bias):
    return [torch.empty_like(x), torch.empty_like(weight), x.new_empty(weight.shape[0] if need_bias else 0)]


def _linear_setup(ctx, inputs, output):
    x, weight, bias, act = inputs
    ctx.save_for_backward(x, weight, output)
    ctx.act, ctx.has_bias = act, bias is not None


def _linear_backward(ctx, dy):
    x, weight, y = ctx.saved_tensors
    dx, dW, db = linear_bwd(x, weight, y, dy, ctx.act, ctx.has_bias)
    return dx, dW, (db if ctx.has_bias else None), None


linear.register_autograd(_linear_backward, setup_context=_linear_setup)


OPS = ("encoder", "encoder_bwd", "sampler", "sampler_bwd", "sampler_sample", "sampler_sample_bwd", "sampler_kl",
       "sampler_kl_bwd", "decoder", "decoder_bwd", "linear", "linear_bwd")


def registered() -> Sequence[str]:
    """Names of the abcd:: operators torch knows about."""
    return [n for n in OPS if hasattr(torch.ops.abcd, n)]
