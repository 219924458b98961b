"""Production-shape fixtures on the CPU: the inputs
regenerate bit-exactly from their seeds, the product's modules initialise to
the reference's weights (init order, learning.py:84-92), and the oracle
reproduces the reference's step at F = 129, H = Hm = D = 256, K = 128 / 1024
(tests/golden/make_golden.py:run_prod wrote the fixtures by importing the
reference).  The GPU side is tests/test_gpu_prod.py."""
import hashlib

import pytest
import torch

from golden_io import PROD, load_prod, prod_inputs, sha16
from oracle import abcd_oracle as O


def prod_cfg(meta):
    d = meta["dims"]
    return O.default_cfg(F=d["F"], H=d["H"], Hdec=d["H"], Hm=d["Hm"], D=d["D"], K=d["K"], rnn=meta["rnn"],
                         plain=meta.get("plain", False), fplain=d["FPLAIN"], num_speakers=d["NSPK"],
                         speaker_dim=d["S"])


def build_product(meta, device="cpu"):
    """The product modules built as Learner does (seed 1111, encoder -> sampler -> decoder)."""
    from modules import model as M
    d = meta["dims"]
    torch.manual_seed(1111)
    enc = M.RNN_Variational_Encoder(d["F"], d["H"], rnn_type=meta["rnn"])
    if meta.get("plain"):
        samp = M.Sampler(enc.hidden_size_total, d["Hm"], d["FPLAIN"])
        fdim = d["FPLAIN"]
    else:
        samp = M.ABCDSampler(enc.hidden_size_total, d["Hm"], d["K"], d["D"])
        fdim = d["D"]
    dec = M.RNN_Variational_Decoder(d["F"], d["H"], d["Hm"], fdim, rnn_type=meta["rnn"], num_speakers=d["NSPK"],
                                    speaker_embed_dim=d["S"])
    for m in (enc, samp, dec):
        m.to(device).train()
    return enc, samp, dec


def module_sha(m):
    h = hashlib.sha256()
    for v in m.state_dict().values():
        h.update(v.detach().contiguous().cpu().numpy().tobytes())
    return h.hexdigest()[:16]


def test_prod_fixtures_present():
    assert {"lstm_k128", "lstm_k128_pretrain", "gru_k1024_spk", "lstm_k1024_spk", "plain_lstm"} <= set(PROD)


@pytest.mark.parametrize("name", PROD)
def test_prod_inputs_regenerate(name):
    meta, _ = load_prod(name)
    inp = prod_inputs(meta)
    for k, h in meta["sha"].items():
        assert sha16(inp[k]) == h, k
    assert int(inp["data"].shape[0]) == meta["L"] and int(inp["batch_sizes"].numel()) == meta["T"]
    assert int(inp["batch_sizes"][0]) == meta["B"] > 64  # two 64-row tile groups


@pytest.mark.parametrize("name", PROD)
def test_product_init_matches_reference(name):
    meta, _ = load_prod(name)
    mods = build_product(meta)
    for pfx, m in zip(("encoder", "feature_sampler", "decoder"), mods):
        assert module_sha(m) == meta["init_sha"][pfx], pfx


@pytest.mark.parametrize("name", PROD)
def test_oracle_prod_step(name):
    meta, arr = load_prod(name)
    cfg = prod_cfg(meta)
    P = O.init_params(cfg, 1111)
    inp = prod_inputs(meta)
    batch = dict(data=inp["data"], batch_sizes=inp["batch_sizes"], is_offset=inp["is_offset"],
                 speakers=inp["speakers"])
    out, grads, new, total, _ = O.train_step(P, batch, cfg, dict(feat=inp["feat_noise"], eps=inp["eps"]), meta["N"],
                                             pretrain=meta.get("pretrain", False), lr=meta["lr"], clip=meta["clip"])
    for k in ("loss", "em", "off", "kl"):
        assert abs(float(out[k]) - float(arr[k])) <= 2e-5 * abs(float(arr[k])) + 1e-5, k
    for k in ("last_hidden", "logits", "feats", "offset_logits"):
        ref = arr[k].double()
        assert (out[k].double() - ref).abs().max() <= 1e-5 * ref.abs().max(), k
    assert abs(total - float(arr["total_norm"])) <= 1e-4 * float(arr["total_norm"])
    if not meta.get("plain"):
        assert torch.equal(out["logits"].argmax(-1), arr["logits"].argmax(-1))
    for k, g in grads.items():
        if "gn/" + k in arr:
            ref = float(arr["gn/" + k])
            assert abs(float(g.double().norm()) - ref) <= 1e-4 * ref + 1e-12, k
        if "g/" + k in arr:
            ref = arr["g/" + k].double()
            assert (g.double() - ref).abs().max() <= 2e-4 * ref.abs().max() + 1e-12, k
