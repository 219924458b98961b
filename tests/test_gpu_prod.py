"""The timed kernels against the reference at production shapes (SURVEY.md
§8c G4).

The fixtures (tests/golden/prod_*.npz) hold one reference training step at
F = 129, H = Hm = D = 256, K = 128 / 1024, speaker 256, LSTM / GRU / plain,
with B = 72 (two 64-row tile groups) and T = 20.  The weights come from the
init order (checked on the CPU in test_prod_fixtures.py), the inputs and
noise from seeds.  Each case runs FusedStep on the default persistent path
and asserts which kernels ran (abcd_dispatch_name), so the template instances
bench.py times at config 2 / 4 / 5 are the ones compared with the reference.

Tolerances: loss terms 1e-4 relative (north star), logits / last hidden 1e-4
of the tensor's max, gradients 1e-3 of the tensor's max (norms 1e-3
relative), post-SGD parameter deltas 1e-3, argmax categories exact."""
import os

import pytest
import torch

from golden_io import PROD, load_prod, prod_inputs
from gpu_helpers import named_params, rel_err
from test_prod_fixtures import build_product

pytestmark = pytest.mark.gpu

LOSS_TOL = 1e-4
GRAD_TOL = 1e-3

# the kernels bench.py's configs dispatch at H = Hm = 256, F = 129 (Fp = 144)
EXPECT = {
    "LSTM": {"enc_fwd": "enc_fwd_persist<4,16,8>", "enc_bwd": "enc_bwd_w8<4>",
             "dec_fwd": "dec_fwd_x6<13,8,8,LSTM>", "dec_bwd": "dec_bwd_w16<9,LSTM>"},
    "GRU": {"enc_fwd": "enc_fwd_persist<3,16,8>", "enc_bwd": "enc_bwd_w8<3>",
            "dec_fwd": "dec_fwd_x6<13,8,8,GRU>", "dec_bwd": "dec_bwd_w16<9,GRU>"},
}


def _noise(inp):
    q = [] if inp["feat_noise"] is None else [inp["feat_noise"]]
    return q + [inp["eps"]]


@pytest.mark.parametrize("name", PROD)
def test_fused_step_prod_vs_reference(name):
    from modules import engine, noise, _native as N
    meta, arr = load_prod(name)
    enc, samp, dec = build_product(meta, "cuda")
    step = engine.FusedStep(enc, samp, dec)
    named = named_params(enc, samp, dec)
    init = {k: p.detach().clone() for k, p in named.items()}
    inp = prod_inputs(meta)
    noise.replay(*_noise(inp))
    N.lib().abcd_dispatch_reset()
    sc, logits = step.forward_backward(inp["data"].cuda(), inp["batch_sizes"], inp["is_offset"].cuda(),
                                       inp["speakers"].cuda(), meta["N"], is_pretraining=meta.get("pretrain", False))
    torch.cuda.synchronize()
    ran = N.dispatch()
    for role, kern in EXPECT[meta["rnn"]].items():
        assert ran[role][0].startswith(kern), (role, ran[role])
        assert ran[role][1] == 1, (role, ran[role])
    # 2 row groups x 32 members (dec_bwd_w16: 3 groups of 32 rows x 16 members)
    assert ran["dec_bwd"][0].endswith("grid 48") and ran["dec_fwd"][0].endswith("grid 64")
    if not meta.get("plain"):  # the fused sampler head, 5 tiles of 16 rows (the last one ragged: 72 = 4 x 16 + 8)
        assert "samp_head_fwd grid 5" in ran["samp_fwd"][0] and ran["samp_fwd"][1] == 1, ran["samp_fwd"]
        assert ran["samp_bwd"][0].startswith("samp_head_bwd grid 5") and ran["samp_bwd"][1] == 1, ran["samp_bwd"]
    sc = sc.cpu()
    for i, k in ((engine.EM, "em"), (engine.OFF, "off"), (engine.KL, "kl"), (engine.LOSS, "loss")):
        ref = float(arr[k])
        assert abs(float(sc[i]) - ref) <= LOSS_TOL * abs(ref) + 1e-5, (k, float(sc[i]), ref)
    assert rel_err(step.last_hidden, arr["last_hidden"]) < 1e-4
    assert rel_err(logits, arr["logits"]) < 1e-4
    assert rel_err(step.feats, arr["feats"]) < 1e-4
    if not meta.get("plain"):
        assert torch.equal(logits.argmax(-1).cpu(), arr["logits"].argmax(-1))
    for k, p in named.items():
        g = step.flat.grad_of(p).detach().double().cpu()
        if "gn/" + k in arr:
            ref = float(arr["gn/" + k])
            assert abs(float(g.norm()) - ref) <= GRAD_TOL * ref + 1e-12, (k, float(g.norm()), ref)
        if "g/" + k in arr:
            assert rel_err(g, arr["g/" + k]) < GRAD_TOL, (k, rel_err(g, arr["g/" + k]))
        if "grow/" + k in arr:
            assert rel_err(g.sum(1), arr["grow/" + k]) < GRAD_TOL, k
            assert rel_err(g.sum(0), arr["gcol/" + k]) < GRAD_TOL, k
    step.optimizer_step(lr=meta["lr"], momentum=0.0, clip=meta["clip"])
    torch.cuda.synchronize()
    assert abs(float(step.scalars[engine.NORM]) - float(arr["total_norm"])) <= 1e-4 * float(arr["total_norm"])
    for k, p in named.items():
        delta = (p.detach().double().cpu() - init[k].double().cpu())
        ref_n, ref_s = float(arr["dq_norm/" + k]), float(arr["dq_sum/" + k])
        assert abs(float(delta.norm()) - ref_n) <= GRAD_TOL * ref_n + 1e-9, (k, float(delta.norm()), ref_n)
        assert abs(float(delta.sum()) - ref_s) <= GRAD_TOL * ref_n * delta.numel() ** 0.5 + 1e-9, k


@pytest.mark.parametrize("name", ["lstm_k128", "gru_k1024_spk", "plain_lstm"])
def test_module_surface_prod_vs_reference(name):
    """encoder(packed) -> sampler -> sample -> kl -> decoder on the nn.Module
    surface at production shapes: the decoder's per-frame outputs (mu, log-var,
    self-fed samples, offset logits) against the reference's row sums."""
    from modules import noise
    meta, arr = load_prod(name)
    enc, samp, dec = build_product(meta, "cuda")
    inp = prod_inputs(meta)
    packed = torch.nn.utils.rnn.PackedSequence(inp["data"].cuda(), inp["batch_sizes"])
    noise.replay(*_noise(inp))
    h = enc(packed)
    if meta.get("plain"):
        fp = samp(h)
        feats = samp.sample(fp)
        kl = samp.kl_divergence(fp)
    else:
        logits = samp(h)
        feats = samp.sample(logits, no_sample=meta.get("pretrain", False))
        kl = samp.kl_divergence(logits, meta["N"])
    em, off, flat, (mu, lv), offl = dec(feats, batch_sizes=inp["batch_sizes"], speaker=inp["speakers"].cuda(),
                                        ground_truth_out=packed.data, ground_truth_offset=inp["is_offset"].cuda())
    loss = (em + off + kl) / meta["B"]
    assert abs(float(loss.detach()) - float(arr["loss"])) <= LOSS_TOL * abs(float(arr["loss"]))
    assert rel_err(mu.sum(1), arr["mu_rowsum"]) < 1e-4
    assert rel_err(lv.sum(1), arr["lv_rowsum"]) < 1e-4
    assert rel_err(flat.sum(1), arr["flat_rowsum"]) < 1e-4
    assert rel_err(mu.sum(0), arr["mu_colsum"]) < 1e-4
    assert rel_err(offl, arr["offset_logits"]) < 1e-4


def test_persist_timeout_is_fatal(monkeypatch):
    """A persistent kernel whose hand-off wait times out (ABCD_SPIN_LIMIT=0
    makes the first unsatisfied poll give up) flags the step's STATUS slot;
    the trainer's read of the records raises instead of training on garbage."""
    from modules import engine, noise, _native as N
    meta, _ = load_prod("lstm_k128")
    enc, samp, dec = build_product(meta, "cuda")
    step = engine.FusedStep(enc, samp, dec)
    inp = prod_inputs(meta)
    args = (inp["data"].cuda(), inp["batch_sizes"], inp["is_offset"].cuda(), inp["speakers"].cuda(), meta["N"])
    assert N.lib().abcd_device_status() == 0
    monkeypatch.setenv("ABCD_SPIN_LIMIT", "0")
    noise.replay(*_noise(inp))
    sc = step.step(*args).clone()
    torch.cuda.synchronize()
    assert float(sc[engine.STATUS]) != 0.0
    with pytest.raises(N.PersistTimeout):
        engine.check_status(torch.stack([torch.zeros_like(sc), sc]).cpu(), "training batch")
    assert N.lib().abcd_device_status() != 0  # sticky until read
    monkeypatch.delenv("ABCD_SPIN_LIMIT")
    noise.replay(*_noise(inp))
    sc = step.step(*args).clone()  # default bound restored on the next launch
    torch.cuda.synchronize()
    assert float(sc[engine.STATUS]) == 0.0
    assert N.lib().abcd_device_status() == 0
    engine.check_status(sc.cpu())


def test_op_surface_timeout_does_not_poison_later_launches(monkeypatch):
    """a hand-off timeout on the op surface (ops.encoder through
    the nn.Module, which never runs FusedStep's status fold) is reported by
    the op-surface probe (PersistTimeout), and the NEXT launch with the
    default spin bound is unaffected: its waits are not abandoned because of
    the earlier launch's timeout (the abort word is per launch), so it
    reproduces the healthy result bit for bit."""
    from modules import _native as N
    meta, _ = load_prod("lstm_k128")
    enc, samp, dec = build_product(meta, "cuda")
    inp = prod_inputs(meta)
    packed = torch.nn.utils.rnn.PackedSequence(inp["data"].cuda(), inp["batch_sizes"])
    N.op_status.sync("setup")
    with torch.no_grad():
        good = enc(packed).clone()
        torch.cuda.synchronize()
        N.op_status.sync("healthy launch")
        monkeypatch.setenv("ABCD_SPIN_LIMIT", "0")
        enc(packed)
        torch.cuda.synchronize()
        with pytest.raises(N.PersistTimeout):
            N.op_status.sync("forced timeout")
        monkeypatch.delenv("ABCD_SPIN_LIMIT")
        again = enc(packed)
        torch.cuda.synchronize()
    N.op_status.sync("launch after the timeouts")
    assert torch.equal(again, good)


def test_fused_step_wide_decoder_separate_offset_head():
    """The offset head's GEMM-folded forms (gemm_x6r8 modes 1 / 2) take a
    decoder hidden size <= 256; a wider decoder (H = 288 here) runs the
    separate head kernels (dec_offset_head / dec_offset_bwd) beside plain
    GEMMs, and the per-step recurrent kernels.  One fused training step
    against the oracle (model.py:287-334 offset MLP + BCE, learning.py:147-163)."""
    from modules import engine, noise
    from modules import model as M
    from oracle import abcd_oracle as O
    F, He, Hd, Hm, D, K = 33, 32, 288, 64, 32, 16
    lengths = [11, 9, 9, 6, 3, 2]
    g = torch.Generator().manual_seed(17)
    seqs = [torch.randn(T, F, generator=g) for T in lengths]
    packed = torch.nn.utils.rnn.pack_sequence(seqs)
    is_off = torch.nn.utils.rnn.pack_sequence([torch.tensor([0.0] * (T - 1) + [1.0]) for T in lengths]).data
    B = len(lengths)
    gumbel = -torch.empty(B, K).exponential_(generator=g).log()
    eps = torch.randn(packed.data.shape[0], F, generator=g)
    torch.manual_seed(1111)
    enc = M.RNN_Variational_Encoder(F, He)
    samp = M.ABCDSampler(enc.hidden_size_total, Hm, K, D)
    dec = M.RNN_Variational_Decoder(F, Hd, Hm, D)
    for m in (enc, samp, dec):
        m.cuda().train()
    ocfg = O.default_cfg(F=F, H=He, Hdec=Hd, Hm=Hm, D=D, K=K)
    P = O.init_params(ocfg, 1111)
    named = named_params(enc, samp, dec)
    for k, p in named.items():
        assert torch.equal(p.detach().cpu(), P[k]), k
    step = engine.FusedStep(enc, samp, dec)
    noise.replay(gumbel, eps)
    sc, _ = step.forward_backward(packed.data.cuda(), packed.batch_sizes, is_off.cuda(), torch.zeros(B).cuda(), 50)
    torch.cuda.synchronize()
    out, grads, _, _, _ = O.train_step(
        P, dict(data=packed.data, batch_sizes=packed.batch_sizes, is_offset=is_off), ocfg,
        dict(feat=gumbel, eps=eps), 50)
    sc = sc.cpu()
    for i, k in ((engine.EM, "em"), (engine.OFF, "off"), (engine.KL, "kl"), (engine.LOSS, "loss")):
        assert abs(float(sc[i]) - float(out[k])) <= 1e-4 * abs(float(out[k])) + 1e-5, (k, float(sc[i]), float(out[k]))
    for k, p in named.items():
        assert rel_err(step.flat.grad_of(p), grads[k]) < GRAD_TOL, (k, rel_err(step.flat.grad_of(p), grads[k]))
