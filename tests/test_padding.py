"""The zero-padded model (seq2seq_abcd-vae_amd/modules/padding.py) on the CPU.

The HIP kernels tile hidden / MLP / feature / category / speaker sizes by 16;
other sizes run as the zero-padded twin.  These tests pin the padding maps
without a GPU:

* every real parameter lands at its unit / gate / block position of the
  twin and every other entry of the twin is 0;
* the padded twin IS the real model: the oracle (torch-CPU restatement of
  the reference step) run on the twin's parameters at the padded sizes gives
  the real model's losses, and its gradients at the real positions are the
  real gradients, while every padding gradient is exactly 0.  (Categories and
  the codebook dim stay multiples of 16 here: the kernels mask padding
  categories and rescale by the real D, which the oracle does not know.)
"""
import itertools

import pytest
import torch

from oracle import abcd_oracle as O

PREFIX = {0: "encoder", 1: "feature_sampler", 2: "decoder"}


def _modules(F, H, Hm, D, K, rnn="LSTM", layers=1, bidir=True, S=None, nspk=None):
    from modules import model as M
    torch.manual_seed(1111)
    enc = M.RNN_Variational_Encoder(F, H, rnn_type=rnn, rnn_layers=layers, bidirectional=bidir)
    samp = M.ABCDSampler(enc.hidden_size_total, Hm, K, D)
    dec = M.RNN_Variational_Decoder(F, H, Hm, D, rnn_type=rnn, num_speakers=nspk, speaker_embed_dim=S)
    return enc, samp, dec


def _named(mods):
    out = {}
    for i, m in enumerate(mods):
        for k, v in m.named_parameters():
            out[f"{PREFIX[i]}/{k}"] = v
    return out


CASES = [dict(F=9, H=24, Hm=40, D=32, K=16, S=12, nspk=3),
         dict(F=9, H=20, Hm=24, D=16, K=16, rnn="GRU", layers=2),
         dict(F=9, H=24, Hm=16, D=16, K=16, bidir=False)]


@pytest.mark.parametrize("case", CASES)
def test_pad_plan_embeds_every_parameter(case):
    from modules import padding as P
    mods = _modules(**case)
    plan = P.PadPlan(*mods)
    real = torch.cat([p.detach().reshape(-1) for m in mods for p in m.parameters()])
    assert plan.index.numel() == real.numel() and plan.index.unique().numel() == real.numel()
    flat = torch.zeros(plan.padded_numel)
    flat.index_copy_(0, plan.index, real)
    assert float(flat.abs().sum()) == pytest.approx(float(real.abs().sum()), rel=1e-6)
    # per parameter: ModulePad's differentiable embedding agrees with the flat map
    off = 0
    for kind, m, twin in zip(("encoder", "sampler", "decoder"), mods, plan.twins):
        tw = dict(twin.named_parameters())
        for name, p in m.named_parameters():
            n = tw[name].numel()
            seg = flat[off:off + n].view(tw[name].shape)
            off += n
            assert seg.abs().sum() == pytest.approx(float(p.detach().abs().sum()), rel=1e-6), name
    assert off == plan.padded_numel


def test_module_pad_matches_plan_for_each_module():
    from modules import padding as P
    mods = _modules(F=9, H=24, Hm=40, D=20, K=10, S=12, nspk=3)
    enc, samp, dec = mods
    me = P.ModulePad("encoder", enc)
    w = me.weights(enc._weights())
    for t, (name, p) in zip(w, enc.named_parameters()):
        assert tuple(t.shape) == tuple(dict(me.twin.named_parameters())[name].shape)
        assert float(t.detach().abs().sum()) == pytest.approx(float(p.detach().abs().sum()), rel=1e-6)
    ms = P.ModulePad("sampler", samp)
    assert ms.cfg[:4] == [P.up16(enc.hidden_size_total), 48, 16, 32] and ms.cfg[5:] == [10, 20]
    md = P.ModulePad("decoder", dec)
    assert md.cfg[1:4] == [32, 48, 32] and md.cfg[7] == 16
    # the embedding is differentiable: gradients reach the real tensor only at its entries
    t = md.weight(dec.feature2hidden.weight)
    t.sum().backward()
    assert torch.equal(dec.feature2hidden.weight.grad, torch.ones_like(dec.feature2hidden.weight))


def _oracle_cfg(F, H, Hm, D, K, rnn="LSTM", layers=1, bidir=True, S=None, nspk=None):
    return O.default_cfg(F=F, H=H, Hdec=H, Hm=Hm, D=D, K=K, rnn=rnn, layers=layers, bidirectional=bidir,
                         num_speakers=nspk, speaker_dim=S)


@pytest.mark.parametrize("case", CASES)
def test_padded_twin_is_the_real_model(case):
    """oracle step on the real parameters == oracle step on the padded twin."""
    from modules import padding as P
    mods = _modules(**case)
    plan = P.PadPlan(*mods)
    g = torch.Generator().manual_seed(5)
    lengths = [7, 5, 5, 3, 2]
    F, K = case["F"], case["K"]
    seqs = [torch.randn(T, F, generator=g) for T in lengths]
    packed = torch.nn.utils.rnn.pack_sequence(seqs)
    is_off = torch.nn.utils.rnn.pack_sequence([torch.tensor([0.0] * (T - 1) + [1.0]) for T in lengths]).data
    B = len(lengths)
    noise = dict(feat=-torch.empty(B, K).exponential_(generator=g).log(),
                 eps=torch.randn(packed.data.shape[0], F, generator=g))
    batch = dict(data=packed.data, batch_sizes=packed.batch_sizes, is_offset=is_off,
                 speakers=torch.randint(0, case.get("nspk") or 1, (B,), generator=g))
    named = _named(mods)
    Preal = {k: v.detach().clone() for k, v in named.items()}
    Preal["feature_sampler/prior_concentration"] = torch.tensor(1.0)
    cfg = _oracle_cfg(**case)
    out_r, grads_r, _, _, _ = O.train_step(Preal, batch, cfg, noise, 50)
    # the twin's parameters from the flat map
    real = torch.cat([p.detach().reshape(-1) for m in mods for p in m.parameters()])
    flat = torch.zeros(plan.padded_numel)
    flat.index_copy_(0, plan.index, real)
    Ppad, off = {}, 0
    for i, twin in enumerate(plan.twins):
        for k, v in twin.named_parameters():
            Ppad[f"{PREFIX[i]}/{k}"] = flat[off:off + v.numel()].view(v.shape).clone()
            off += v.numel()
    Ppad["feature_sampler/prior_concentration"] = torch.tensor(1.0)
    de, ds, dd = plan.dims
    pcase = dict(case, H=de.Hp, Hm=ds.Hmp, S=(dd.Sp or None))
    out_p, grads_p, _, _, _ = O.train_step(Ppad, batch, _oracle_cfg(**pcase), noise, 50)
    for k in ("em", "off", "kl", "loss"):
        assert float(out_p[k]) == pytest.approx(float(out_r[k]), rel=1e-5), k
    assert torch.allclose(out_p["logits"], out_r["logits"], atol=1e-5)
    gr = torch.cat([grads_r[k].reshape(-1) for k in named])
    gp = torch.cat([grads_p[k].reshape(-1) for k in Ppad if k in grads_p])
    mask = torch.zeros(plan.padded_numel, dtype=torch.bool)
    mask[plan.index] = True
    assert torch.allclose(gp[plan.index], gr, rtol=1e-4, atol=1e-6 * float(gr.abs().max()))
    assert float(gp[~mask].abs().max()) == 0.0  # padding weights receive exactly no gradient
