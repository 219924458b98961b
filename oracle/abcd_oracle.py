"""CPU oracle for the ABCD-VAE training step -- TEST INFRASTRUCTURE ONLY.

This module is the *checker*.  It is imported only by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg; the
product path (``seq2seq_abcd-vae_amd/``) never imports, links or executes it.

It restates, in plain torch-CPU fp32 tensor arithmetic (matmul + elementwise,
autograd for the backward), the algorithm of the reference hot path
``ABCD-VAE/learning.py:147-163`` as it is spread over the reference files:

* encoder   ``ABCD-VAE/modules/model.py:40-66``  (``torch.nn.LSTM/GRU`` over a
  PackedSequence -- the recurrence itself lives in third-party torch
  2.10.0+rocm7.0, whose published LSTM/GRU equations are restated below)
* sampler   ``model.py:538-639`` (ABCD) / ``plain/modules/model.py:538-567``
* decoder   ``model.py:84-196,262-300``, emission ``model.py:17-37,676-705``
* step      ``learning.py:147-163`` (loss / batch_sizes[0], backward,
  ``clip_grad_norm_``, ``SGD``)
* init      ``learning.py:84-92`` + the torch ``reset_parameters`` of
  ``nn.LSTM/GRU/LSTMCell/GRUCell/Linear/Embedding``.

Parity of this restatement is PINNED by ``tests/golden/*.npz`` and
``tests/golden/toy_known_answers.json``, which were produced by importing the
reference itself (``tests/golden/make_golden.py``); ``tests/test_oracle.py``
checks the oracle against every one of them.
"""
import math
from collections import OrderedDict

import torch

LOG2PI = math.log(2 * math.pi)


# ----------------------------------------------------------------------------
# configuration helpers
# ----------------------------------------------------------------------------
def default_cfg(**kw):
    cfg = dict(F=129, H=256, Hdec=256, Hm=256, D=256, K=128, rnn="LSTM", dec_rnn=None,
               layers=1, bidirectional=True, greedy=False, plain=False, fplain=16,
               num_speakers=None, speaker_dim=None, prior_concentration=1.0)
    cfg.update(kw)
    if cfg["dec_rnn"] is None:
        cfg["dec_rnn"] = cfg["rnn"]
    return cfg


def encoder_out_size(cfg):
    e = cfg["layers"] * cfg["H"] * (2 if cfg["bidirectional"] else 1)
    return e * 2 if cfg["rnn"] == "LSTM" else e


# ----------------------------------------------------------------------------
# init (restates learning.py:84-92 module construction order and torch's
# reset_parameters for each layer type)
# ----------------------------------------------------------------------------
def _uniform(shape, bound):
    return torch.empty(shape).uniform_(-bound, bound)


def _linear(fan_in, fan_out):
    # torch.nn.Linear.reset_parameters: kaiming_uniform_(a=sqrt(5)) then bias U(-1/sqrt(fan_in), .)
    gain = math.sqrt(2.0 / (1 + 5.0))
    std = gain / math.sqrt(fan_in)
    w = _uniform((fan_out, fan_in), math.sqrt(3.0) * std)
    b = _uniform((fan_out,), 1.0 / math.sqrt(fan_in))
    return w, b


def init_params(cfg, seed=1111):
    """Parameters in the reference's state_dict order; same torch RNG calls in
    the same order as ``Learner.__init__`` (learning.py:84-92)."""
    torch.manual_seed(seed)
    P = OrderedDict()
    F, H, Hm, D, K = cfg["F"], cfg["H"], cfg["Hm"], cfg["D"], cfg["K"]
    G = 4 if cfg["rnn"] == "LSTM" else 3
    dirs = ["", "_reverse"] if cfg["bidirectional"] else [""]
    stdv = 1.0 / math.sqrt(H)
    # nn.LSTM/GRU: every parameter U(-1/sqrt(H), 1/sqrt(H)) in _flat_weights order
    for l in range(cfg["layers"]):
        In = F if l == 0 else H * len(dirs)
        for sfx in dirs:
            P[f"encoder/rnn.weight_ih_l{l}{sfx}"] = _uniform((G * H, In), stdv)
            P[f"encoder/rnn.weight_hh_l{l}{sfx}"] = _uniform((G * H, H), stdv)
            P[f"encoder/rnn.bias_ih_l{l}{sfx}"] = _uniform((G * H,), stdv)
            P[f"encoder/rnn.bias_hh_l{l}{sfx}"] = _uniform((G * H,), stdv)
    E = encoder_out_size(cfg)
    if cfg["plain"]:
        f = cfg["fplain"]
        for k in range(2):
            w1, b1 = _linear(E, Hm); w2, b2 = _linear(Hm, f)
            pre = f"feature_sampler/to_parameters.mlps.{k}.whole_network"
            P[f"{pre}.0.weight"], P[f"{pre}.0.bias"] = w1, b1
            P[f"{pre}.2.weight"], P[f"{pre}.2.bias"] = w2, b2
        feat = f
    else:
        w1, b1 = _linear(E, Hm); w2, b2 = _linear(Hm, D)
        psl = torch.randn(K)
        cb = torch.randn(D, K)
        # state_dict order: own parameters, own buffers, then children (model.py:555-579)
        P["feature_sampler/posterior_shape_logits"] = psl
        P["feature_sampler/codebook"] = cb
        P["feature_sampler/prior_concentration"] = torch.tensor(float(cfg["prior_concentration"]))
        P["feature_sampler/to_code_like.whole_network.0.weight"] = w1
        P["feature_sampler/to_code_like.whole_network.0.bias"] = b1
        P["feature_sampler/to_code_like.whole_network.2.weight"] = w2
        P["feature_sampler/to_code_like.whole_network.2.bias"] = b2
        feat = D
    Hd = cfg["Hdec"]
    Gd = 4 if cfg["dec_rnn"] == "LSTM" else 3
    htot = 2 * Hd if cfg["dec_rnn"] == "LSTM" else Hd
    if cfg["num_speakers"] is not None and cfg["speaker_dim"] is not None:
        P["decoder/embed_speaker.weight"] = torch.randn(cfg["num_speakers"], cfg["speaker_dim"])
        feat += cfg["speaker_dim"]
    P["decoder/feature2hidden.weight"], P["decoder/feature2hidden.bias"] = _linear(feat, htot)
    w1, b1 = _linear(Hd, Hm); w2, b2 = _linear(Hm, 1)
    P["decoder/offset_predictor.whole_network.0.weight"], P["decoder/offset_predictor.whole_network.0.bias"] = w1, b1
    P["decoder/offset_predictor.whole_network.2.weight"], P["decoder/offset_predictor.whole_network.2.bias"] = w2, b2
    for k in range(2):
        w1, b1 = _linear(Hd, Hm); w2, b2 = _linear(Hm, F)
        pre = f"decoder/emission_sampler.to_parameters.mlps.{k}.whole_network"
        P[f"{pre}.0.weight"], P[f"{pre}.0.bias"] = w1, b1
        P[f"{pre}.2.weight"], P[f"{pre}.2.bias"] = w2, b2
    s = 1.0 / math.sqrt(Hd)
    P["decoder/rnn_cell.cell.weight_ih"] = _uniform((Gd * Hd, F), s)
    P["decoder/rnn_cell.cell.weight_hh"] = _uniform((Gd * Hd, Hd), s)
    P["decoder/rnn_cell.cell.bias_ih"] = _uniform((Gd * Hd,), s)
    P["decoder/rnn_cell.cell.bias_hh"] = _uniform((Gd * Hd,), s)
    return P


def is_buffer(name):
    return name.endswith("prior_concentration")


# ----------------------------------------------------------------------------
# recurrent cells (PyTorch's published equations; gate order i,f,g,o / r,z,n)
# ----------------------------------------------------------------------------
def lstm_cell(x, h, c, W_ih, W_hh, b_ih, b_hh):
    g = x @ W_ih.t() + b_ih + h @ W_hh.t() + b_hh
    i, f, gg, o = g.chunk(4, 1)
    i, f, gg, o = torch.sigmoid(i), torch.sigmoid(f), torch.tanh(gg), torch.sigmoid(o)
    c = f * c + i * gg
    return o * torch.tanh(c), c


def gru_cell(x, h, W_ih, W_hh, b_ih, b_hh):
    gi = x @ W_ih.t() + b_ih
    gh = h @ W_hh.t() + b_hh
    ir, iz, inn = gi.chunk(3, 1)
    hr, hz, hn = gh.chunk(3, 1)
    r = torch.sigmoid(ir + hr)
    z = torch.sigmoid(iz + hz)
    n = torch.tanh(inn + r * hn)
    return (1 - z) * n + z * h


def _offsets(batch_sizes):
    off = [0]
    for bs in batch_sizes[:-1]:
        off.append(off[-1] + int(bs))
    return off


def rnn_layer_packed(x, batch_sizes, w, rnn, reverse):
    """One direction of one layer over packed (time-major) rows.
    Returns (outputs L x H in packed order, final h (B x H), final c or None)."""
    bsz = [int(b) for b in batch_sizes]
    off = _offsets(bsz)
    T, B = len(bsz), bsz[0]
    H = w[1].shape[1]
    outs = [None] * T
    fin_h = [None] * B
    fin_c = [None] * B
    order = range(T - 1, -1, -1) if reverse else range(T)
    h = c = None
    for t in order:
        bs = bsz[t]
        xt = x[off[t]:off[t] + bs]
        if h is None:
            h = x.new_zeros(bs, H); c = x.new_zeros(bs, H)
        elif h.shape[0] > bs:          # forward: sequences ended -> shrink
            h, c = h[:bs], c[:bs]
        elif h.shape[0] < bs:          # reverse: sequences start -> grow with zeros
            pad = bs - h.shape[0]
            h = torch.cat([h, x.new_zeros(pad, H)], 0); c = torch.cat([c, x.new_zeros(pad, H)], 0)
        if rnn == "LSTM":
            h, c = lstm_cell(xt, h, c, *w)
        else:
            h = gru_cell(xt, h, *w)
        outs[t] = h
        if not reverse:
            nxt = bsz[t + 1] if t + 1 < T else 0
            for b in range(nxt, bs):
                fin_h[b] = h[b]; fin_c[b] = c[b] if rnn == "LSTM" else None
    if reverse:
        fin_h = list(h); fin_c = list(c) if rnn == "LSTM" else [None] * B
    out = torch.cat(outs, 0)
    fh = torch.stack(fin_h, 0)
    fc = torch.stack(fin_c, 0) if rnn == "LSTM" else None
    return out, fh, fc


def encoder_forward(P, data, batch_sizes, cfg):
    """model.py:60-66: returns last_hidden (B x hidden_size_total) laid out as
    transpose(cat(h_n, c_n, -1), 0, 1).view(B, -1)."""
    dirs = ["", "_reverse"] if cfg["bidirectional"] else [""]
    x = data
    pieces = []
    for l in range(cfg["layers"]):
        outs = []
        for sfx in dirs:
            w = [P[f"encoder/rnn.{n}_l{l}{sfx}"] for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
            out, fh, fc = rnn_layer_packed(x, batch_sizes, w, cfg["rnn"], reverse=(sfx == "_reverse"))
            outs.append(out)
            pieces.append(torch.cat([fh, fc], -1) if cfg["rnn"] == "LSTM" else fh)
        x = torch.cat(outs, -1)
    return torch.cat(pieces, -1)


def mlp(x, P, pre):
    h = torch.tanh(x @ P[f"{pre}.0.weight"].t() + P[f"{pre}.0.bias"])
    return h @ P[f"{pre}.2.weight"].t() + P[f"{pre}.2.bias"]


# ----------------------------------------------------------------------------
# ABCD sampler (model.py:581-639) and plain Gaussian sampler (plain model.py)
# ----------------------------------------------------------------------------
def abcd_logits(P, h):
    u = mlp(h, P, "feature_sampler/to_code_like.whole_network")
    return u @ P["feature_sampler/codebook"] / math.sqrt(u.shape[-1])


def abcd_sample(P, logits, gumbel=None, tau=1.0):
    """pretrain (gumbel None): softmax(logits); else softmax((logits+g)/tau)
    with g = -log(Exp(1)) (F.gumbel_softmax, hard=False)."""
    if gumbel is None:
        y = torch.softmax(logits, -1)
    else:
        y = torch.softmax((logits + gumbel) / tau, -1)
    return y @ P["feature_sampler/codebook"].t()


def digamma_kl(P, logits, N):
    psl = P["feature_sampler/posterior_shape_logits"]
    a0 = P["feature_sampler/prior_concentration"]
    K = psl.shape[0]
    alpha = torch.softmax(psl, -1) * N + a0
    S = alpha.sum()
    elog = torch.digamma(alpha) - torch.digamma(S)
    eq_log_q_pi = torch.lgamma(S) - torch.lgamma(alpha).sum() + ((alpha - 1.0) * elog).sum()
    eq_log_p_pi = torch.lgamma(a0 * K) - torch.lgamma(a0) * K + ((a0 - 1.0) * elog).sum()
    q = torch.softmax(logits, -1)
    logq = torch.log_softmax(logits, -1)
    B = logits.shape[0]
    return (eq_log_q_pi - eq_log_p_pi) * (B / N) + (q * logq).sum() - (q * elog[None, :]).sum()


def plain_params(P, h):
    mu = mlp(h, P, "feature_sampler/to_parameters.mlps.0.whole_network")
    lv = mlp(h, P, "feature_sampler/to_parameters.mlps.1.whole_network")
    return mu, lv


def gaussian_kl(mu, lv):
    return -0.5 * (1 + lv - mu.pow(2) - lv.exp()).sum()


# ----------------------------------------------------------------------------
# decoder (model.py:147-196)
# ----------------------------------------------------------------------------
def decoder_forward(P, feats, batch_sizes, cfg, eps, speakers=None, gt=None, gt_off=None, train=True, xmask=None):
    bsz = [int(b) for b in batch_sizes]
    Hd = cfg["Hdec"]
    F = cfg["F"]
    if "decoder/embed_speaker.weight" in P:
        feats = torch.cat([feats, P["decoder/embed_speaker.weight"][speakers]], -1)
    hid = feats @ P["decoder/feature2hidden.weight"].t() + P["decoder/feature2hidden.bias"]
    lstm = cfg["dec_rnn"] == "LSTM"
    if lstm:
        hid = hid.view(-1, Hd, 2)
        h, c = hid[..., 0], hid[..., 1]
    else:
        h, c = hid.view(-1, Hd), None
    w = [P[f"decoder/rnn_cell.cell.{n}"] for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
    x = feats.new_zeros(bsz[0], F)
    feedback = not (cfg["greedy"] and train)
    off = _offsets(bsz)
    hs, mus, lvs, outs = [], [], [], []
    for t, bs in enumerate(bsz):
        xin = x[:bs] if feedback else x[:bs] * 0.0
        if xmask is not None and train:  # RNN_Cell input dropout, model.py:297 (noise bernoulli(1-p)/(1-p))
            xin = xin * xmask[off[t]:off[t] + bs]
        if lstm:
            h, c = lstm_cell(xin, h[:bs], c[:bs], *w)
        else:
            h = gru_cell(xin, h[:bs], *w)
        mu = mlp(h, P, "decoder/emission_sampler.to_parameters.mlps.0.whole_network")
        lv = mlp(h, P, "decoder/emission_sampler.to_parameters.mlps.1.whole_network")
        x = mu + (0.5 * lv).exp() * eps[off[t]:off[t] + bs]
        hs.append(h); mus.append(mu); lvs.append(lv); outs.append(x)
    H_all = torch.cat(hs, 0); MU = torch.cat(mus, 0); LV = torch.cat(lvs, 0); OUT = torch.cat(outs, 0)
    off_logits = mlp(H_all, P, "decoder/offset_predictor.whole_network").squeeze(-1)
    em = off_loss = None
    if gt is not None:
        d = gt - MU
        em = 0.5 * (LOG2PI + LV + d * (-LV).exp() * d).sum()
    if gt_off is not None:
        off_loss = torch.nn.functional.binary_cross_entropy_with_logits(off_logits, gt_off, reduction="sum")
    return em, off_loss, OUT, (MU, LV), off_logits


# ----------------------------------------------------------------------------
# one training step (learning.py:147-163)
# ----------------------------------------------------------------------------
def forward_losses(P, batch, cfg, noise, N, pretrain=False, tau=1.0, train=True, loss_batch=None):
    data, batch_sizes = batch["data"], batch["batch_sizes"]
    last_hidden = encoder_forward(P, data, batch_sizes, cfg)
    if cfg["plain"]:
        mu_f, lv_f = plain_params(P, last_hidden)
        feats = mu_f + (0.5 * lv_f).exp() * noise["feat"]
        kl = gaussian_kl(mu_f, lv_f)
        logits = torch.cat([mu_f, lv_f], -1)
    else:
        logits = abcd_logits(P, last_hidden)
        feats = abcd_sample(P, logits, None if pretrain else noise["feat"], tau)
        kl = digamma_kl(P, logits, N)
    em, off, out, (mu, lv), off_logits = decoder_forward(
        P, feats, batch_sizes, cfg, noise["eps"], speakers=batch.get("speakers"),
        gt=data, gt_off=batch["is_offset"], train=train, xmask=noise.get("xmask"))
    # learning.py:156 divides by batch_sizes[0]; a data-parallel shard divides
    # by the global batch size instead (loss_batch), so the ranks' losses sum
    # to the global-batch loss
    B = int(batch_sizes[0]) if loss_batch is None else int(loss_batch)
    loss = (em + off + kl) / B
    return dict(loss=loss, em=em, off=off, kl=kl, last_hidden=last_hidden, logits=logits, feats=feats,
                flatten_out=out, mu=mu, lv=lv, offset_logits=off_logits)


def train_step(P, batch, cfg, noise, N, pretrain=False, tau=1.0, lr=1.0, clip=1.0,
               momentum=0.0, momentum_buf=None, loss_batch=None):
    """Returns (outputs, grads, new_params, total_norm, momentum_buf)."""
    P = OrderedDict((k, v.detach().clone().requires_grad_(not is_buffer(k))) for k, v in P.items())
    out = forward_losses(P, batch, cfg, noise, N, pretrain, tau, loss_batch=loss_batch)
    out["loss"].backward()
    names = [k for k in P if not is_buffer(k)]
    grads = OrderedDict((k, P[k].grad.detach().clone() if P[k].grad is not None else torch.zeros_like(P[k]))
                        for k in names)
    # torch.nn.utils.clip_grad_norm_ (total 2-norm, coef = clip/(norm+1e-6), clamp 1)
    total = torch.sqrt(sum((g.double() ** 2).sum() for g in grads.values())).float()
    coef = torch.clamp(clip / (total + 1e-6), max=1.0)
    new = OrderedDict()
    mbuf = OrderedDict() if momentum_buf is None else momentum_buf
    for k, v in P.items():
        if is_buffer(k):
            new[k] = v.detach().clone()
            continue
        g = grads[k] * coef
        if momentum != 0.0:
            if k in mbuf:
                mbuf[k] = mbuf[k] * momentum + g
            else:
                mbuf[k] = g.clone()
            g = mbuf[k]
        new[k] = (v.detach() - lr * g)
    out = {k: (v.detach() if torch.is_tensor(v) else v) for k, v in out.items()}
    return out, grads, new, float(total), mbuf


def perplexities(logits, psl):
    """learning.py:171-178 diagnostics."""
    p = torch.softmax(logits, -1)
    cl = (-p * p.log()).sum(-1).mean().exp()
    bm = p.mean(0); bm = bm / bm.sum()
    bp = (-bm * bm.log()).sum().exp()
    ps = torch.softmax(psl, -1)
    sp = (-ps * ps.log()).sum().exp()
    return float(cl), float(bp), float(sp)
