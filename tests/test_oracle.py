"""The CPU oracle against the reference's own outputs (golden fixtures).

These are the tests that PIN the oracle: every fixture was produced by
importing /root/reference (tests/golden/make_golden.py)."""
import hashlib

import pytest
import torch

from golden_io import SMALL, load_small, small_cfg, params_from, batch_from, noise_from, load_toy, known_answers
from oracle import abcd_oracle as O


def close(a, b, rtol, atol_frac=1e-5):
    a = a.double(); b = b.double()
    scale = max(b.abs().max().item(), 1e-30)
    err = (a - b).abs().max().item()
    assert err <= rtol * scale + atol_frac * scale, f"maxerr {err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("name", SMALL)
def test_oracle_small_step(name):
    meta, arr = load_small(name)
    cfg = small_cfg(meta)
    P = params_from(arr)
    out, grads, new, total, _ = O.train_step(
        P, batch_from(arr), cfg, noise_from(meta, arr), meta["N"], pretrain=meta.get("pretrain", False),
        tau=meta.get("temperature") or 1.0, lr=meta["lr"], clip=meta["clip"])
    for k in ("loss", "em", "off", "kl"):
        assert abs(float(out[k]) - float(arr[k])) <= 2e-5 * abs(float(arr[k])) + 1e-5, k
    for k in ("last_hidden", "logits", "feats", "flatten_out", "mu", "lv", "offset_logits"):
        close(out[k], arr[k], 1e-5)
    assert abs(total - float(arr["total_norm"])) <= 1e-4 * float(arr["total_norm"])
    for k, g in grads.items():
        if "g/" + k in arr:
            close(g, arr["g/" + k], 2e-4)
    for k, v in new.items():
        close(v, arr["q/" + k], 1e-5)


@pytest.mark.parametrize("name", SMALL)
def test_oracle_init_order(name):
    """init_params restates the reference's construction order (learning.py:84-92)."""
    meta, arr = load_small(name)
    cfg = small_cfg(meta)
    P = O.init_params(cfg, 1111)
    ref = params_from(arr)
    assert list(P.keys()) == list(ref.keys())
    for k in P:
        assert torch.equal(P[k], ref[k]), k


def test_oracle_toy_init_checksums():
    cks, toy = load_toy()
    cfg = O.default_cfg(F=65, K=16)
    P = O.init_params(cfg, 1111)
    for mod in ("encoder", "feature_sampler", "decoder"):
        vals = [v for k, v in P.items() if k.startswith(mod + "/")]
        h = hashlib.sha256()
        for v in vals:
            h.update(v.contiguous().numpy().tobytes())
        assert h.hexdigest()[:16] == cks[mod][1], mod
        assert abs(sum(float(v.double().sum()) for v in vals) - cks[mod][0]) < 1e-6
    assert torch.equal(P["feature_sampler/codebook"][0, :4], toy["codebook_0_4"])


def test_oracle_toy_first_batch():
    """Full-width toy step (F=65, H=256, K=16): first batch of epoch 1 of config 1."""
    _, toy = load_toy()
    cfg = O.default_cfg(F=65, K=16)
    P = O.init_params(cfg, 1111)
    batch = dict(data=toy["data"], batch_sizes=toy["batch_sizes"], is_offset=toy["is_offset"])
    out, grads, new, total, _ = O.train_step(P, batch, cfg, dict(feat=None, eps=toy["eps"]), int(toy["N"]),
                                             pretrain=True)
    ka = known_answers()["lstm_softmax_e2"]
    assert abs(float(out["loss"]) - ka["batch_loss"][0]) <= 1e-5 * ka["batch_loss"][0]
    for k in ("em", "off", "kl"):
        assert abs(float(out[k]) - float(toy[k])) <= 1e-5 * abs(float(toy[k])) + 1e-4, k
    close(out["logits"], toy["logits"], 1e-5)
    close(out["last_hidden"], toy["last_hidden"], 1e-5)
    for k, g in grads.items():
        ref = float(toy["gn/" + k])
        assert abs(g.norm().item() - ref) <= 1e-4 * ref + 1e-6, k
    assert abs(total - float(toy["total_norm"])) <= 1e-4 * float(toy["total_norm"])
