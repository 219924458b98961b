"""HIP path vs the reference's own outputs (golden fixtures) and the oracle.

Every case runs through libabcd_hip.so (C ABI).  Tolerances: losses 1e-4
relative (north-star bar: reconstruction loss <= 1e-4), gradients 1e-3 of the
tensor's max magnitude (fp32 MFMA reduction order vs torch CPU), post-SGD
parameters 1e-5 relative, argmax categories exact."""
import pytest
import torch

from golden_io import SMALL, load_small, small_cfg, params_from, batch_from, noise_from
from gpu_helpers import build_from_meta, named_params, rel_err

pytestmark = pytest.mark.gpu

LOSS_TOL = 1e-4
GRAD_TOL = 1e-3


def _noise_list(meta, arr):
    q = []
    if meta.get("plain") or not meta.get("pretrain", False):
        q.append(arr["feat_noise"])
    q.append(arr["eps"])
    if "xmask" in arr:  # decoder input dropout: replayed after eps (noise.decoder_noise)
        q.append(arr["xmask"])
    return q


@pytest.fixture(scope="module")
def modules_pkg():
    from modules import engine, noise, model  # noqa
    return engine, noise, model


@pytest.mark.parametrize("name", SMALL)
def test_fused_step_vs_reference(name, modules_pkg):
    engine, noise, _ = modules_pkg
    meta, arr = load_small(name)
    enc, samp, dec = build_from_meta(meta, arr)
    step = engine.FusedStep(enc, samp, dec)
    b = batch_from(arr)
    noise.replay(*_noise_list(meta, arr))
    sc, logits = step.forward_backward(b["data"].cuda(), b["batch_sizes"], b["is_offset"].cuda(),
                                       b["speakers"].cuda(), meta["N"], is_pretraining=meta.get("pretrain", False))
    torch.cuda.synchronize()
    sc = sc.cpu()
    for i, k in ((engine.EM, "em"), (engine.OFF, "off"), (engine.KL, "kl"), (engine.LOSS, "loss")):
        ref = float(arr[k])
        assert abs(float(sc[i]) - ref) <= LOSS_TOL * abs(ref) + 1e-5, (k, float(sc[i]), ref)
    assert rel_err(logits, arr["logits"]) < 1e-4
    named = named_params(enc, samp, dec)
    for k, p in named.items():
        g = step.flat.grad_of(p)
        ref = arr["g/" + k]
        assert rel_err(g, ref) < GRAD_TOL, (k, rel_err(g, ref))
    step.optimizer_step(lr=meta["lr"], momentum=0.0, clip=meta["clip"])
    torch.cuda.synchronize()
    assert abs(float(step.scalars[engine.NORM]) - float(arr["total_norm"])) <= 1e-4 * float(arr["total_norm"])
    for k, p in named.items():
        assert rel_err(p, arr["q/" + k]) < 1e-5, k


@pytest.mark.parametrize("name", ["lstm_gumbel", "gru_gumbel", "lstm_speaker", "plain_lstm", "lstm_2layer",
                                  "lstm_ddrop", "lstm_odd", "gru_odd_2layer", "plain_odd"])
def test_module_autograd_vs_reference(name, modules_pkg):
    """The nn.Module surface (encoder(packed) -> sampler -> sample -> kl ->
    decoder -> loss.backward()) on the HIP autograd Functions."""
    engine, noise, _ = modules_pkg
    meta, arr = load_small(name)
    enc, samp, dec = build_from_meta(meta, arr)
    b = batch_from(arr)
    packed = torch.nn.utils.rnn.PackedSequence(b["data"].cuda(), b["batch_sizes"])
    noise.replay(*_noise_list(meta, arr))
    h = enc(packed)
    assert rel_err(h, arr["last_hidden"]) < 1e-4
    if meta.get("plain"):
        fp = samp(h)
        feats = samp.sample(fp)
        kl = samp.kl_divergence(fp)
    else:
        logits = samp(h)
        feats = samp.sample(logits, no_sample=meta.get("pretrain", False))
        kl = samp.kl_divergence(logits, meta["N"])
    assert rel_err(feats, arr["feats"]) < 1e-4
    em, off, flat, (mu, lv), offl = dec(feats, batch_sizes=b["batch_sizes"], speaker=b["speakers"].cuda(),
                                        ground_truth_out=packed.data, ground_truth_offset=b["is_offset"].cuda())
    loss = (em + off + kl) / int(b["batch_sizes"][0])
    loss.backward()
    assert abs(float(loss) - float(arr["loss"])) <= LOSS_TOL * abs(float(arr["loss"]))
    assert rel_err(flat, arr["flatten_out"]) < 1e-4
    assert rel_err(mu, arr["mu"]) < 1e-4
    assert rel_err(offl, arr["offset_logits"]) < 1e-4
    for k, p in named_params(enc, samp, dec).items():
        assert p.grad is not None, k
        g = p.grad.to_dense() if p.grad.is_sparse else p.grad
        assert rel_err(g, arr["g/" + k]) < GRAD_TOL, (k, rel_err(g, arr["g/" + k]))
