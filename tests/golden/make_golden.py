#!/usr/bin/env python3
"""Generate the golden fixtures that pin ``oracle/`` (and, through it, the HIP path).

TEST INFRASTRUCTURE ONLY.  This script is the one place that imports the
upstream reference (``/root/reference``, read-only).  It runs in the build
container only; nothing under ``tests/`` reads ``/root/reference`` at test time
and the reference never travels to the GPU box -- only the ``.npz`` / ``.json``
outputs written next to this file do.

Nothing in the reference is edited.  Four compatibility shims are applied to
the *imported module objects* so that a PyTorch-1.2-era codebase runs on torch
2.10:

1. ``Dataset.get_discrete_bounds``: pandas 2 keeps ``onset_ix/offset_ix`` as
   float64 -> cast to ``int`` (``ABCD-VAE/modules/data_utils.py:69-79``).
2. ``STFT.__call__``: ``Tensor.stft`` now needs ``return_complex``; the
   complex result is turned into the same real-pair amplitude
   (``data_utils.py:131-139``).
3. ``torch._six.inf`` (``learning.py:285``).
4. ``clip_grad_norm_`` on a sparse speaker-embedding grad (torch-1.2 style
   per-parameter norm over coalesced values) -- only matters with
   ``--speaker_embed_dim``.

Fixtures written (all small, committed):

* ``small_<variant>.npz``  one full training step (fwd, loss, bwd, clip, SGD)
  at reduced widths, with the replayed noise, every parameter, every output,
  every gradient and every post-SGD parameter.  Variants cover LSTM/GRU,
  softmax (pretrain) vs Gumbel, speaker embedding, 2-layer and
  unidirectional encoders, greedy decoder, temperature < 1 and the plain
  Gaussian VAE.
* ``toy_step.npz``          the first training batch of the toy config
  (``toy_data``, ``-b 4 -K 16``, F=65, H=256) at full widths: inputs, losses,
  logits, gradient norms per parameter, init checksums.
* ``toy_known_answers.json`` loss trajectories of the reference CLI on the toy
  data (config 1 of BASELINE.json and its variants) and the ``encode.py``
  argmax per segment.
* ``prod_<variant>.npz``    one training step at the production widths of
  BASELINE.json configs 2/4/5 (F=129, H=Hm=D=256, K=128/1024, speaker 256,
  LSTM/GRU/plain) with B=72 (two 64-row tile groups): outputs, loss terms,
  gradient norms / full small gradients / row+column sums of the large ones,
  post-SGD deltas.  Weights come from the init order, inputs and noise from
  seeds (``tests/golden_io.py:prod_inputs``).
* ``ref_ckpt_small.pt`` + ``ref_ckpt_small_encode.npz``  a checkpoint written
  by the reference CLI (small widths, toy data, 1 epoch) and the reference
  ``encode.py``'s probabilities for it.

* ``ref_ckpt_plain.pt`` + ``ref_plain_encode{,_named}.csv``  a plain-VAE
  checkpoint written by plain/learning.py and plain/encode.py's tables for it.

Usage: ``python tests/golden/make_golden.py [--only small|prod|toy|cli|ckpt|ckpt_plain]``.
"""
import argparse
import hashlib
import json
import math
import os
import re
import subprocess
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------
# shims (applied to the imported reference module objects, never to files)
# --------------------------------------------------------------------------
def apply_shims(data_utils, torch):
    orig_bounds = data_utils.Dataset.get_discrete_bounds

    def get_discrete_bounds(self):
        orig_bounds(self)
        for col in ("onset_ix", "offset_ix", "length"):
            self.df_annotation[col] = self.df_annotation[col].astype(int)

    data_utils.Dataset.get_discrete_bounds = get_discrete_bounds

    def stft_call(self, input_data):
        z = input_data.stft(self.frame_length, hop_length=self.step_size, window=self.window,
                            center=self.centering, return_complex=True)
        return torch.view_as_real(z).pow(2).sum(-1).sqrt().transpose(0, 1).contiguous()

    data_utils.STFT.__call__ = stft_call
    torch._six = types.SimpleNamespace(inf=math.inf)

    def clip_grad_norm_legacy(parameters, max_norm, norm_type=2):
        parameters = [p for p in parameters if p.grad is not None]
        total = 0.0
        for p in parameters:
            g = p.grad.data
            if g.is_sparse:
                g = g.coalesce()._values()
            total += g.norm(norm_type).item() ** norm_type
        total = total ** (1.0 / norm_type)
        coef = max_norm / (total + 1e-6)
        if coef < 1:
            for p in parameters:
                if p.grad.is_sparse:
                    # `p.grad.data.mul_` on a sparse grad is not seen by the
                    # optimizer on torch 2.x (it was on 1.2): scale explicitly
                    p.grad = p.grad.coalesce() * coef
                else:
                    p.grad.data.mul_(coef)
        return total

    return clip_grad_norm_legacy


def import_reference(variant_dir):
    import torch
    sys.path.insert(0, os.path.join(REF, variant_dir))
    from modules import model, data_utils  # noqa: E402  (reference, read-only)
    clip = apply_shims(data_utils, torch)
    return torch, model, data_utils, clip


# --------------------------------------------------------------------------
# small one-step fixtures
# --------------------------------------------------------------------------
SMALL_LENGTHS = [12, 10, 10, 7, 4, 2]
SMALL_DIMS = dict(F=33, H=32, Hm=32, D=32, K=16, S=16, NSPK=3, FPLAIN=16)

SMALL_VARIANTS = {
    "lstm_gumbel": dict(rnn="LSTM"),
    "lstm_pretrain": dict(rnn="LSTM", pretrain=True),
    "lstm_tau": dict(rnn="LSTM", tau=0.7),
    "gru_gumbel": dict(rnn="GRU"),
    "lstm_speaker": dict(rnn="LSTM", speaker=True),
    "lstm_2layer": dict(rnn="LSTM", layers=2),
    "lstm_uni": dict(rnn="LSTM", bidirectional=False),
    "lstm_greedy": dict(rnn="LSTM", greedy=True),
    "lstm_ddrop": dict(rnn="LSTM", input_dropout=0.3),
    "gru_speaker_pretrain": dict(rnn="GRU", speaker=True, pretrain=True),
    "plain_lstm": dict(rnn="LSTM", plain=True),
    "plain_gru": dict(rnn="GRU", plain=True),
    # sizes that are not multiples of 16 (the HIP path runs the zero-padded
    # model, seq2seq_abcd-vae_amd/modules/padding.py): K = 10, H = 24, Hm = 40,
    # D = 20, speaker dim 12; a 2-layer GRU at H = 20; the plain VAE at f = 10
    "lstm_odd": dict(rnn="LSTM", speaker=True, dims=dict(H=24, Hm=40, D=20, K=10, S=12)),
    "gru_odd_2layer": dict(rnn="GRU", layers=2, dims=dict(H=20, Hm=24, D=12, K=10)),
    "plain_odd": dict(rnn="LSTM", plain=True, dims=dict(H=24, Hm=40, FPLAIN=10)),
}


def state_items(prefix, module):
    return {f"{prefix}/{k}": v.detach().clone() for k, v in module.state_dict().items()}


def run_small(name, cfg):
    plain = cfg.get("plain", False)
    torch, model, data_utils, clip_legacy = import_reference("plain" if plain else "ABCD-VAE")
    d = dict(SMALL_DIMS, **cfg.get("dims", {}))
    F, H, Hm, D, K = d["F"], d["H"], d["Hm"], d["D"], d["K"]
    rnn = cfg["rnn"]
    layers = cfg.get("layers", 1)
    bidir = cfg.get("bidirectional", True)
    speaker = cfg.get("speaker", False)
    greedy = cfg.get("greedy", False)
    pretrain = cfg.get("pretrain", False)
    p_in = cfg.get("input_dropout", 0.0)
    nspk = d["NSPK"] if speaker else None
    sdim = d["S"] if speaker else None
    N_total = 50  # entire_data_size

    # -------- data (own generator: does not touch the global RNG) --------
    gen = torch.Generator().manual_seed(20240611)
    seqs = [2.0 * torch.randn(T, F, generator=gen) - 1.0 for T in SMALL_LENGTHS]
    spk = torch.randint(0, d["NSPK"], (len(SMALL_LENGTHS),), generator=gen)
    packed = torch.nn.utils.rnn.pack_sequence(seqs)
    is_offset = torch.nn.utils.rnn.pack_sequence(
        [torch.tensor([0.0] * (len(s) - 1) + [1.0]) for s in seqs])
    batch_sizes = packed.batch_sizes
    B = int(batch_sizes[0])

    # -------- model, init order as Learner.__init__ (learning.py:84-92) --------
    torch.manual_seed(1111)
    enc = model.RNN_Variational_Encoder(F, H, rnn_type=rnn, rnn_layers=layers,
                                        hidden_dropout=0.0, bidirectional=bidir)
    if plain:
        samp = model.Sampler(enc.hidden_size_total, Hm, d["FPLAIN"])
        feat_dim = d["FPLAIN"]
    else:
        samp = model.ABCDSampler(enc.hidden_size_total, Hm, K, D)
        feat_dim = D
        if "tau" in cfg:
            samp.temperature = cfg["tau"]
    dec = model.RNN_Variational_Decoder(F, H, Hm, feat_dim, rnn_type=rnn,
                                        self_feedback=not greedy, input_dropout=p_in,
                                        num_speakers=nspk, speaker_embed_dim=sdim)
    modules = [("encoder", enc), ("feature_sampler", samp), ("decoder", dec)]
    out = {}
    for p, m in modules:
        out.update({"p/" + k: v for k, v in state_items(p, m).items()})
    enc.train(); samp.train(); dec.train()

    # -------- noise replay (verified bit-exact) --------
    state = torch.get_rng_state()
    if plain:
        feat_noise = torch.randn(B, feat_dim)
    elif not pretrain:
        feat_noise = -torch.empty(B, K).exponential_().log()
    else:
        feat_noise = torch.zeros(0)
    if p_in > 0.0:
        # RNN_Cell's dropout of step t's input (model.py:297), then the
        # sampler's randn (model.py:19), per step
        masks, epss = [], []
        for bs in batch_sizes:
            masks.append(torch.empty(int(bs), F).bernoulli_(1 - p_in).div_(1 - p_in))
            epss.append(torch.randn(int(bs), F))
        xmask, eps = torch.cat(masks, 0), torch.cat(epss, 0)
    else:
        xmask, eps = None, torch.cat([torch.randn(int(bs), F) for bs in batch_sizes], 0)
    torch.set_rng_state(state)

    # -------- the Learner.train step body (learning.py:147-163) --------
    params = list(enc.parameters()) + list(samp.parameters()) + list(dec.parameters())
    opt = torch.optim.SGD(params, lr=1.0, momentum=0.0)
    opt.zero_grad()
    last_hidden = enc(packed)
    if plain:
        fparams = samp(last_hidden)
        feats = samp.sample(fparams)
        kl = samp.kl_divergence(fparams)
        logits = torch.cat(fparams, -1)
    else:
        logits = samp(last_hidden)
        feats = samp.sample(logits, no_sample=pretrain)
        kl = samp.kl_divergence(logits, N_total)
    em, off, flat_out, (mu, lv), off_logits = dec(
        feats, batch_sizes=batch_sizes, speaker=spk if speaker else torch.full((B,), float("nan")),
        ground_truth_out=packed.data, ground_truth_offset=is_offset.data)
    loss = (em + off + kl) / batch_sizes[0]
    loss.backward()
    grads = {}
    for p, m in modules:
        for k, v in m.named_parameters():
            g = v.grad
            if g is None:
                continue
            if g.is_sparse:
                g = g.to_dense()
            grads[f"g/{p}/{k}"] = g.detach().clone()
    if speaker:
        total_norm = clip_legacy(params, 1.0)
    else:
        total_norm = float(torch.nn.utils.clip_grad_norm_(params, 1.0))
    opt.step()
    for p, m in modules:
        out.update({"q/" + k: v for k, v in state_items(p, m).items()})

    # reproduce check: the replayed noise is what the reference consumed
    if not plain:
        assert torch.allclose(flat_out, mu + (0.5 * lv).exp() * eps, atol=1e-5, rtol=1e-5)

    out.update({
        "data": packed.data, "batch_sizes": batch_sizes, "is_offset": is_offset.data,
        "speakers": spk, "feat_noise": feat_noise, "eps": eps,
        "last_hidden": last_hidden, "logits": logits, "feats": feats,
        "kl": kl, "em": em, "off": off, "loss": loss, "flatten_out": flat_out,
        "mu": mu, "lv": lv, "offset_logits": off_logits,
        "total_norm": torch.tensor(total_norm),
    })
    if xmask is not None:
        out["xmask"] = xmask
    out.update(grads)
    meta = dict(cfg, name=name, dims=d, N=N_total, lengths=SMALL_LENGTHS, lr=1.0, clip=1.0,
                temperature=(None if plain else samp.temperature))
    arrays = {k: (v.detach().numpy() if hasattr(v, "detach") else np.asarray(v)) for k, v in out.items()}
    arrays = {k: v.astype(np.float32) if v.dtype == np.float64 else v for k, v in arrays.items()}
    arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    path = os.path.join(HERE, f"small_{name}.npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path}: loss={float(loss):.6f} em={float(em):.4f} off={float(off):.4f} kl={float(kl):.6f}")


# --------------------------------------------------------------------------
# production-shape one-step fixtures
# --------------------------------------------------------------------------
# Widths of BASELINE.json configs 2/4/5 (F = 129, H = Hm = D = 256, K = 128 or
# 1024, speaker 256) with B = 72 segments, so the persistent kernels run two
# 64-row tile groups (the second one 8 rows, all short), and T <= 24 so the
# reference finishes in seconds.  Weights are NOT stored: they are re-created
# by the init order (torch.manual_seed(1111), encoder -> sampler -> decoder)
# and pinned by per-module checksums.  Inputs and noise are regenerated from
# seeds by tests/golden_io.py:prod_inputs (sha256 stored).
PROD_DIMS = dict(F=129, H=256, Hm=256, D=256, K=128, S=None, NSPK=None, FPLAIN=16)
PROD_VARIANTS = {
    "lstm_k128": dict(rnn="LSTM"),
    "lstm_k128_pretrain": dict(rnn="LSTM", pretrain=True),
    "gru_k1024_spk": dict(rnn="GRU", K=1024, S=256, NSPK=16),
    "lstm_k1024_spk": dict(rnn="LSTM", K=1024, S=256, NSPK=16),
    "plain_lstm": dict(rnn="LSTM", plain=True),
}
FULL_GRAD_MAX = 40000  # gradients up to this many elements are stored in full


def run_prod(name, cfg):
    plain = cfg.get("plain", False)
    torch, model, data_utils, clip_legacy = import_reference("plain" if plain else "ABCD-VAE")
    sys.path.insert(0, os.path.dirname(HERE))
    from golden_io import prod_inputs, sha16  # noqa: E402  (build-owned helper)
    d = dict(PROD_DIMS, **{k: cfg[k] for k in ("K", "S", "NSPK") if k in cfg})
    meta = dict(cfg, name=name, dims=d, B=72, tmin=4, tmax=20, seed_data=4242, seed_noise=777, N=10000,
                lr=1.0, clip=1.0)
    F, H, Hm, D, K = d["F"], d["H"], d["Hm"], d["D"], d["K"]
    rnn, pretrain, speaker = cfg["rnn"], cfg.get("pretrain", False), d["NSPK"] is not None
    inp = prod_inputs(meta)
    B = meta["B"]

    torch.manual_seed(1111)
    enc = model.RNN_Variational_Encoder(F, H, rnn_type=rnn)
    if plain:
        samp = model.Sampler(enc.hidden_size_total, Hm, d["FPLAIN"])
        fdim = d["FPLAIN"]
    else:
        samp = model.ABCDSampler(enc.hidden_size_total, Hm, K, D)
        fdim = D
    dec = model.RNN_Variational_Decoder(F, H, Hm, fdim, rnn_type=rnn, num_speakers=d["NSPK"],
                                        speaker_embed_dim=d["S"])
    modules = [("encoder", enc), ("feature_sampler", samp), ("decoder", dec)]
    init = {f"{p}/{k}": v.detach().clone() for p, m in modules for k, v in m.state_dict().items()}
    meta["init_sha"] = {p: module_checksums(torch, m)[1] for p, m in modules}
    meta["init_sum"] = {p: module_checksums(torch, m)[0] for p, m in modules}
    enc.train(); samp.train(); dec.train()

    # the reference draws its noise from the global generator: seed it so the
    # draws are exactly prod_inputs' generator stream (checked below)
    torch.manual_seed(meta["seed_noise"])
    packed = torch.nn.utils.rnn.PackedSequence(inp["data"], inp["batch_sizes"])
    params = list(enc.parameters()) + list(samp.parameters()) + list(dec.parameters())
    opt = torch.optim.SGD(params, lr=1.0, momentum=0.0)
    opt.zero_grad()
    last_hidden = enc(packed)
    if plain:
        fparams = samp(last_hidden)
        feats = samp.sample(fparams)
        kl = samp.kl_divergence(fparams)
        logits = torch.cat(fparams, -1)
    else:
        logits = samp(last_hidden)
        feats = samp.sample(logits, no_sample=pretrain)
        kl = samp.kl_divergence(logits, meta["N"])
    spk = inp["speakers"] if speaker else torch.full((B,), float("nan"))
    em, off, flat_out, (mu, lv), off_logits = dec(
        feats, batch_sizes=inp["batch_sizes"], speaker=spk, ground_truth_out=inp["data"],
        ground_truth_offset=inp["is_offset"])
    loss = (em + off + kl) / inp["batch_sizes"][0]
    loss.backward()
    # the replayed noise is what the reference consumed
    assert torch.equal(flat_out, mu + (0.5 * lv).exp() * inp["eps"]) or \
        torch.allclose(flat_out, mu + (0.5 * lv).exp() * inp["eps"], rtol=1e-6, atol=1e-6)
    if not plain and not pretrain:
        y = torch.softmax((logits + inp["feat_noise"]) / samp.temperature, -1)
        assert torch.allclose(feats, y @ samp.codebook.t(), rtol=1e-5, atol=1e-6)
    out = {"last_hidden": last_hidden, "logits": logits, "feats": feats, "kl": kl, "em": em, "off": off,
           "loss": loss, "offset_logits": off_logits,
           "mu_rowsum": mu.sum(1), "lv_rowsum": lv.sum(1), "flat_rowsum": flat_out.sum(1),
           "mu_colsum": mu.sum(0), "lv_colsum": lv.sum(0)}
    for p, m in modules:
        for k, v in m.named_parameters():
            g = v.grad
            if g is None:
                continue
            g = g.to_dense() if g.is_sparse else g
            out[f"gn/{p}/{k}"] = g.norm()
            if g.numel() <= FULL_GRAD_MAX:
                out[f"g/{p}/{k}"] = g.clone()
            elif g.dim() == 2:
                out[f"grow/{p}/{k}"] = g.sum(1)
                out[f"gcol/{p}/{k}"] = g.sum(0)
    total_norm = clip_legacy(params, 1.0) if speaker else float(torch.nn.utils.clip_grad_norm_(params, 1.0))
    opt.step()
    for p, m in modules:
        for k, v in m.state_dict().items():
            delta = (v.detach() - init[f"{p}/{k}"]).double()
            out[f"dq_sum/{p}/{k}"] = delta.sum()
            out[f"dq_norm/{p}/{k}"] = delta.norm()
    out["total_norm"] = torch.tensor(total_norm)
    if not plain:
        top2 = logits.topk(2, -1).values
        meta["argmax_min_gap"] = float((top2[:, 0] - top2[:, 1]).min())
    meta["sha"] = {k: sha16(inp[k]) for k in ("data", "eps", "speakers", "is_offset")}
    if inp["feat_noise"] is not None:
        meta["sha"]["feat_noise"] = sha16(inp["feat_noise"])
    meta["L"] = int(inp["data"].shape[0])
    meta["T"] = int(inp["batch_sizes"].numel())
    meta["temperature"] = None if plain else samp.temperature
    arrays = {k: v.detach().numpy() for k, v in out.items()}
    arrays = {k: v.astype(np.float32) if v.dtype == np.float64 and not k.startswith("dq_") else v
              for k, v in arrays.items()}
    arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    path = os.path.join(HERE, f"prod_{name}.npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path}: L={meta['L']} T={meta['T']} loss={float(loss):.6f} em={float(em):.4f} "
          f"off={float(off):.4f} kl={float(kl):.6f} gap={meta.get('argmax_min_gap')}")


# --------------------------------------------------------------------------
# toy first-batch fixture at full widths (config 1)
# --------------------------------------------------------------------------
def module_checksums(torch, module):
    sd = module.state_dict()
    total = float(sum(v.double().sum() for v in sd.values()))
    h = hashlib.sha256()
    for v in sd.values():
        h.update(v.detach().contiguous().numpy().tobytes())
    return total, h.hexdigest()[:16]


def run_toy_step():
    torch, model, data_utils, _ = import_reference("ABCD-VAE")
    root = os.path.join(REF, "toy_data")
    ann = os.path.join(root, "annotation_20170806-080002_89.2-94.22.csv")
    parser = data_utils.Data_Parser(root, ann)
    fs = parser.get_sample_freq()
    frame = int(np.floor(0.008 * fs)); step = int(np.floor(0.004 * fs))
    F = int(frame / 2 + 1)
    tfm = data_utils.Compose([data_utils.ToTensor(), data_utils.STFT(frame, step),
                              data_utils.Transform(lambda x: (x + 2 ** (-15)).log() / 1.0)])
    train = parser.get_data(data_type="train", transform=tfm)
    torch.manual_seed(1111)
    enc = model.RNN_Variational_Encoder(F, 256, rnn_type="LSTM")
    samp = model.ABCDSampler(enc.hidden_size_total, 256, 16, 256)
    dec = model.RNN_Variational_Decoder(F, 256, 256, 256, rnn_type="LSTM")
    cks = {n: module_checksums(torch, m) for n, m in
           [("encoder", enc), ("feature_sampler", samp), ("decoder", dec)]}
    # first batch of epoch 1 exactly as Learner.learn draws it (RandomSampler, pop from end)
    loader = data_utils.DataLoader(train, batch_size=4, shuffle=True)
    it = iter(loader)
    packed, is_offset, spk, ixs = next(it)
    params = list(enc.parameters()) + list(samp.parameters()) + list(dec.parameters())
    state = torch.get_rng_state()
    eps = torch.cat([torch.randn(int(bs), F) for bs in packed.batch_sizes], 0)
    torch.set_rng_state(state)
    last_hidden = enc(packed)
    logits = samp(last_hidden)
    feats = samp.sample(logits, no_sample=True)
    kl = samp.kl_divergence(logits, len(train))
    em, off, flat_out, (mu, lv), _ = dec(feats, batch_sizes=packed.batch_sizes, speaker=spk,
                                         ground_truth_out=packed.data, ground_truth_offset=is_offset.data)
    loss = (em + off + kl) / packed.batch_sizes[0]
    loss.backward()
    gnorms = {}
    for pfx, m in [("encoder", enc), ("feature_sampler", samp), ("decoder", dec)]:
        for k, v in m.named_parameters():
            gnorms[f"gn/{pfx}/{k}"] = v.grad.norm().detach()
    total_norm = float(torch.nn.utils.clip_grad_norm_(params, 1.0))
    arrays = {
        "data": packed.data, "batch_sizes": packed.batch_sizes, "is_offset": is_offset.data,
        "ixs": torch.as_tensor(np.asarray(ixs)), "eps": eps, "last_hidden": last_hidden, "logits": logits,
        "feats": feats, "kl": kl, "em": em, "off": off, "loss": loss, "mu": mu, "lv": lv,
        "total_norm": torch.tensor(total_norm), "N": torch.tensor(len(train)),
    }
    arrays.update(gnorms)
    arrays = {k: v.detach().numpy() for k, v in arrays.items()}
    arrays["checksums"] = np.frombuffer(json.dumps(cks).encode(), dtype=np.uint8)
    arrays["codebook_0_4"] = samp.codebook.detach()[0, :4].numpy()
    path = os.path.join(HERE, "toy_step.npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path}: loss={float(loss):.4f} em={float(em):.4f} checksums={cks}")


# --------------------------------------------------------------------------
# CLI trajectories on toy data (config 1 and variants)
# --------------------------------------------------------------------------
CLI_RUNS = {
    "lstm_softmax_e2": ("ABCD-VAE", ["-e", "2", "-b", "4", "-R", "LSTM", "-K", "16"]),
    "lstm_gumbel_e2": ("ABCD-VAE", ["-e", "2", "-b", "4", "-R", "LSTM", "-K", "16", "--pretrain_epochs", "0"]),
    "gru_softmax_e2": ("ABCD-VAE", ["-e", "2", "-b", "4", "-R", "GRU", "-K", "16"]),
    "greedy_e2": ("ABCD-VAE", ["-e", "2", "-b", "4", "-R", "LSTM", "-K", "16", "--greedy_decoder"]),
    "plain_e2": ("plain", ["-e", "2", "-b", "4"]),
    "lstm2_drop_e2": ("ABCD-VAE", ["-e", "2", "-b", "4", "-R", "LSTM", "-K", "16", "--encoder_rnn_layers", "2",
                                   "--encoder_hidden_dropout", "0.1"]),
    "ddrop_e2": ("ABCD-VAE", ["-e", "2", "-b", "4", "-R", "LSTM", "-K", "16", "--decoder_input_dropout", "0.3"]),
    # sizes off the 16-grid: one softmax epoch, then Gumbel
    "odd_sizes_e2": ("ABCD-VAE", ["-e", "2", "-b", "4", "-R", "LSTM", "-K", "10", "-f", "20", "--mlp_hidden_size",
                                  "100", "--encoder_rnn_hidden_size", "40", "--decoder_rnn_hidden_size", "24",
                                  "--speaker_embed_dim", "12", "--pretrain_epochs", "1"]),
}

LINE_PATTERNS = {
    "batch_loss": re.compile(r"training batches complete\. mean loss: (-?\d+\.\d+)"),
    "perplex": re.compile(r"clustering probs\.: (-?\d+\.\d+)\. .*minibatch: (-?\d+\.\d+)\. .*shape: (-?\d+\.\d+)"),
    "train_em": re.compile(r"mean training emission negative pdf loss \(per string\): (-?\d+\.\d+)"),
    "train_off": re.compile(r"mean training end-prediction loss \(per string\): (-?\d+\.\d+)"),
    "train_kl": re.compile(r"mean training KL \(per string\): (-?\d+\.\d+)"),
    "train_total": re.compile(r"mean training total loss \(per string\): (-?\d+\.\d+)"),
    "valid_em": re.compile(r"mean validation emission negative pdf loss \(per string\): (-?\d+\.\d+)"),
    "valid_off": re.compile(r"mean validation end-prediction loss \(per string\): (-?\d+\.\d+)"),
    "valid_kl": re.compile(r"mean validation KL \(per string\): (-?\d+\.\d+)"),
    "valid_total": re.compile(r"mean validation total loss \(per string\): (-?\d+\.\d+)"),
}


def parse_history(path):
    res = {k: [] for k in LINE_PATTERNS}
    for line in open(path):
        for k, pat in LINE_PATTERNS.items():
            m = pat.search(line)
            if m:
                vals = [float(x) for x in m.groups()]
                res[k].append(vals if len(vals) > 1 else vals[0])
    return res


def cli_child(variant_dir, script, argv):
    """Run one reference CLI script in this (child) process with the shims."""
    import runpy
    torch, model, data_utils, clip = import_reference(variant_dir)
    torch.set_num_threads(8)
    torch.nn.utils.clip_grad_norm_ = clip
    sys.argv = [script] + argv
    os.chdir(os.path.join(REF, variant_dir))
    runpy.run_path(os.path.join(REF, variant_dir, script), run_name="__main__")


def run_cli(only=None):
    root = os.path.join(REF, "toy_data")
    ann = os.path.join(root, "annotation_20170806-080002_89.2-94.22.csv")
    path = os.path.join(HERE, "toy_known_answers.json")
    results = {}
    if only and os.path.isfile(path):  # refresh one case, keep the others
        with open(path) as f:
            results = json.load(f)
    with tempfile.TemporaryDirectory() as tmp:
        for name, (vdir, flags) in CLI_RUNS.items():
            if only and name != only:
                continue
            save_root = os.path.join(tmp, name)
            cmd = [sys.executable, __file__, "--child", vdir, "learning.py", "--",
                   root, ann, "-S", save_root, "-j", "run"] + flags
            subprocess.run(cmd, check=True)
            hist = parse_history(os.path.join(save_root, "run", "history.log"))
            results[name] = {"flags": flags, **hist}
            print(name, hist["train_total"], hist["valid_total"])
            if name == "lstm_softmax_e2":
                csv = os.path.join(tmp, "encoded.csv")
                ecmd = [sys.executable, __file__, "--child", vdir, "encode.py", "--",
                        os.path.join(save_root, "run", "checkpoint.pt"), root, ann, "1.0",
                        "-S", csv, "-b", "4"]
                subprocess.run(ecmd, check=True)
                import pandas as pd
                df = pd.read_csv(csv)
                df["category_ix"] = df["category_ix"].astype(int)
                best = df.loc[df.groupby("data_ix")["prob"].idxmax()].sort_values("data_ix")
                results[name]["encode_argmax"] = {int(a): int(b) for a, b in
                                                  zip(best["data_ix"], best["category_ix"])}
                results[name]["encode_maxprob"] = {int(a): float(b) for a, b in
                                                   zip(best["data_ix"], best["prob"])}
    with open(path, "w") as f:
        json.dump(results, f, indent=1, sort_keys=True)
    print("wrote", path)


CKPT_FLAGS = ["-e", "1", "-b", "4", "-R", "LSTM", "-K", "16", "-f", "32", "--encoder_rnn_hidden_size", "32",
              "--decoder_rnn_hidden_size", "32", "--mlp_hidden_size", "32", "--pretrain_epochs", "0"]


def run_ckpt():
    """A checkpoint.pt WRITTEN BY THE REFERENCE CLI (learning.py:293-314) at
    small widths on the toy data (weights + optimizer / scheduler state + CPU
    RNG state only: loadable with torch.load(weights_only=True)), and what the
    reference's encode.py makes of it: per-segment probabilities over the K
    categories (the long CSV folded to an 8 x K matrix)."""
    import shutil
    import pandas as pd
    root = os.path.join(REF, "toy_data")
    ann = os.path.join(root, "annotation_20170806-080002_89.2-94.22.csv")
    with tempfile.TemporaryDirectory() as tmp:
        save_root = os.path.join(tmp, "ckpt")
        subprocess.run([sys.executable, __file__, "--child", "ABCD-VAE", "learning.py", "--", root, ann, "-S",
                        save_root, "-j", "run"] + CKPT_FLAGS, check=True)
        ckpt = os.path.join(save_root, "run", "checkpoint.pt")
        shutil.copy(ckpt, os.path.join(HERE, "ref_ckpt_small.pt"))
        csv = os.path.join(tmp, "enc.csv")
        subprocess.run([sys.executable, __file__, "--child", "ABCD-VAE", "encode.py", "--", ckpt, root, ann, "1.0",
                        "-S", csv, "-b", "4"], check=True)
        df = pd.read_csv(csv)
    df["category_ix"] = df["category_ix"].astype(int)
    n, k = int(df["data_ix"].max()) + 1, int(df["category_ix"].max()) + 1
    probs = np.zeros((n, k), np.float32)
    probs[df["data_ix"].to_numpy(), df["category_ix"].to_numpy()] = df["prob"].to_numpy()
    cols = [c for c in df.columns if c not in ("data_ix", "category_ix", "prob")]
    np.savez_compressed(os.path.join(HERE, "ref_ckpt_small_encode.npz"), probs=probs,
                        argmax=probs.argmax(1).astype(np.int64), row_order=df["data_ix"].to_numpy()[:16],
                        meta=np.frombuffer(json.dumps({"flags": CKPT_FLAGS, "columns": list(df.columns),
                                                       "annotation_columns": cols}).encode(), dtype=np.uint8))
    print("wrote ref_ckpt_small.pt / ref_ckpt_small_encode.npz", probs.argmax(1))


PLAIN_CKPT_FLAGS = ["-e", "1", "-b", "4", "-R", "LSTM", "-f", "8", "--encoder_rnn_hidden_size", "32",
                    "--decoder_rnn_hidden_size", "32", "--mlp_hidden_size", "32"]


def run_ckpt_plain():
    """A plain-VAE checkpoint.pt written by the reference CLI
    (plain/learning.py) on the toy data at small widths, and the tables the
    reference's plain/encode.py writes for it: without parameter names
    (-b 3) and with ``-p mean,log_variance`` (-b 4).  The CSVs are the
    reference's output files as written (data: data_ix, parameter_name,
    feature_dim, parameter_value + the annotation columns)."""
    import shutil
    root = os.path.join(REF, "toy_data")
    ann = os.path.join(root, "annotation_20170806-080002_89.2-94.22.csv")
    with tempfile.TemporaryDirectory() as tmp:
        save_root = os.path.join(tmp, "ckpt")
        subprocess.run([sys.executable, __file__, "--child", "plain", "learning.py", "--", root, ann, "-S",
                        save_root, "-j", "run"] + PLAIN_CKPT_FLAGS, check=True)
        ckpt = os.path.join(save_root, "run", "checkpoint.pt")
        shutil.copy(ckpt, os.path.join(HERE, "ref_ckpt_plain.pt"))
        for out, extra in (("ref_plain_encode.csv", ["-b", "3"]),
                           ("ref_plain_encode_named.csv", ["-b", "4", "-p", "mean,log_variance"])):
            subprocess.run([sys.executable, __file__, "--child", "plain", "encode.py", "--", ckpt, root, ann, "1.0",
                            "-S", os.path.join(HERE, out)] + extra, check=True)
    print("wrote ref_ckpt_plain.pt / ref_plain_encode*.csv")


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        vdir, script = sys.argv[2], sys.argv[3]
        cli_child(vdir, script, sys.argv[5:])
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["small", "prod", "toy", "cli", "ckpt", "ckpt_plain"], default=None)
    ap.add_argument("--variant", default=None)
    ap.add_argument("--case", default=None, help="cli: regenerate only this trajectory")
    a = ap.parse_args()
    if not os.path.isdir(REF):
        sys.exit("reference not present; fixtures are committed, nothing to do")
    if a.only in (None, "small"):
        for name, cfg in SMALL_VARIANTS.items():
            if a.variant and name != a.variant:
                continue
            # each variant in its own process: the two reference variants both
            # define a top-level package called `modules`
            subprocess.run([sys.executable, "-c",
                            "import sys; sys.argv=['x']; sys.path.insert(0, %r); import make_golden as m; "
                            "m.run_small(%r, m.SMALL_VARIANTS[%r])" % (HERE, name, name)], check=True)
    if a.only in (None, "prod"):
        for name, cfg in PROD_VARIANTS.items():
            if a.variant and name != a.variant:
                continue
            subprocess.run([sys.executable, "-c",
                            "import sys; sys.argv=['x']; sys.path.insert(0, %r); import make_golden as m; "
                            "m.run_prod(%r, m.PROD_VARIANTS[%r])" % (HERE, name, name)], check=True)
    if a.only in (None, "toy"):
        subprocess.run([sys.executable, "-c",
                        "import sys; sys.path.insert(0, %r); import make_golden as m; m.run_toy_step()" % HERE],
                       check=True)
    if a.only in (None, "cli"):
        run_cli(a.case)
    if a.only in (None, "ckpt"):
        run_ckpt()
    if a.only in (None, "ckpt_plain"):
        run_ckpt_plain()


if __name__ == "__main__":
    main()
