"""End-to-end: the trainer CLI (learning.py) on the reference's toy data vs the
reference CLI's own logged numbers (config 1 of BASELINE.json), and the
encode.py argmax categories after training (bit-exact).

The noise is drawn in the reference's order from torch's CPU generator
(--noise reference), so both runs see identical random numbers; the residual
difference is fp32 summation order (GPU MFMA vs CPU ATen), compounded over the
run's SGD steps."""
import os
import re

import pandas as pd
import pytest
import torch

from golden_io import GOLDEN, known_answers

pytestmark = pytest.mark.gpu

TOY = os.path.join(GOLDEN, "toy_data")
ANN = os.path.join(TOY, "annotation_20170806-080002_89.2-94.22.csv")


def _run(tmp_path, flags, job):
    import learning
    args = [TOY, ANN, "-S", str(tmp_path), "-j", job, "--noise", "reference"] + flags
    learner = learning.main(args)
    return learner, os.path.join(str(tmp_path), job)


def _rel(a, b):
    return abs(a - b) / abs(b)


@pytest.mark.parametrize("case,tol", [("lstm_softmax_e2", 1e-4), ("lstm_gumbel_e2", 1e-4), ("gru_softmax_e2", 1e-4),
                                      ("greedy_e2", 1e-4), ("lstm2_drop_e2", 1e-4), ("ddrop_e2", 1e-4),
                                      ("odd_sizes_e2", 1e-4)])
def test_toy_trajectory_matches_reference(tmp_path, case, tol):
    ka = known_answers()[case]
    learner, save = _run(tmp_path, ka["flags"], case)
    hist = learner.history
    for e in range(2):
        assert _rel(hist[e]["train"]["total"], ka["train_total"][e]) < tol, (e, hist[e]["train"], ka)
        assert _rel(hist[e]["valid"]["total"], ka["valid_total"][e]) < tol, (e, hist[e]["valid"], ka)
        assert _rel(hist[e]["train"]["em"], ka["train_em"][e]) < tol
        assert _rel(hist[e]["valid"]["em"], ka["valid_em"][e]) < tol
    losses = [x for e in range(2) for x in hist[e]["train"]["batch_loss"]]
    for a, b in zip(losses, ka["batch_loss"]):
        assert _rel(a, b) < tol
    if ka.get("perplex"):
        pp = [x for e in range(2) for x in hist[e]["train"]["perplex"]]
        for a, b in zip(pp, ka["perplex"]):
            for x, y in zip(a, b):
                assert abs(x - y) <= 1e-3 * abs(y) + 1e-3
    # history.log carries the reference's lines
    log = open(os.path.join(save, "history.log")).read()
    assert "mean training total loss (per string)" in log
    assert "training batches complete. mean loss:" in log


def test_toy_encode_argmax_matches_reference(tmp_path):
    ka = known_answers()["lstm_softmax_e2"]
    learner, save = _run(tmp_path, ka["flags"], "enc")
    import encode
    out = encode.main([os.path.join(save, "checkpoint.pt"), TOY, ANN, "1.0", "-S",
                       os.path.join(str(tmp_path), "encoded.csv"), "-b", "4"])
    df = pd.read_csv(out)
    best = df.loc[df.groupby("data_ix")["prob"].idxmax()].sort_values("data_ix")
    got = {int(a): int(b) for a, b in zip(best["data_ix"], best["category_ix"])}
    assert got == {int(k): v for k, v in ka["encode_argmax"].items()}


def test_resume_reproduces_uninterrupted_run(tmp_path):
    """learning.py:17-20,317-347: a run resumed from checkpoint.pt continues
    exactly like an uninterrupted one (RNG + optimizer + scheduler state)."""
    ka = known_answers()["lstm_softmax_e2"]
    flags = [f for f in ka["flags"]]
    e_idx = flags.index("-e")
    full_flags = flags[:e_idx + 1] + ["3"] + flags[e_idx + 2:]
    full, _ = _run(tmp_path / "a", full_flags, "run")
    _run(tmp_path / "b", flags, "run")  # 2 epochs
    resumed, _ = _run(tmp_path / "b", full_flags, "run")  # history.log exists -> resume, epoch 3
    assert len(resumed.history) == 1
    assert _rel(resumed.history[0]["train"]["total"], full.history[2]["train"]["total"]) < 1e-6
    assert _rel(resumed.history[0]["valid"]["total"], full.history[2]["valid"]["total"]) < 1e-6


def test_plain_cli_smoke(tmp_path):
    """plain/ Gaussian-VAE trainer on the toy data vs the reference's logged totals."""
    import plain_learning
    ka = known_answers()["plain_e2"]
    learner = plain_learning.main([TOY, ANN, "-S", str(tmp_path), "-j", "plain", "--noise", "reference"] + ka["flags"])
    for e in range(2):
        assert _rel(learner.history[e]["train"]["total"], ka["train_total"][e]) < 1e-4
        assert _rel(learner.history[e]["valid"]["total"], ka["valid_total"][e]) < 1e-4


def test_reference_checkpoint_encodes_like_reference(tmp_path):
    """learning.py:293-347 interop: a checkpoint.pt WRITTEN BY THE REFERENCE CLI
    (tests/golden/ref_ckpt_small.pt, make_golden.py:run_ckpt) is opened by
    retrieve_model (torch.load weights_only=True) and encode.py reproduces the
    reference encode.py's per-segment category probabilities (<= 1e-5) and
    argmax (exact), in the reference's CSV layout."""
    import numpy as np
    import encode
    z = np.load(os.path.join(GOLDEN, "ref_ckpt_small_encode.npz"), allow_pickle=False)
    import json
    meta = json.loads(bytes(z["meta"]).decode())
    out = encode.main([os.path.join(GOLDEN, "ref_ckpt_small.pt"), TOY, ANN, "1.0", "-S",
                       os.path.join(str(tmp_path), "enc.csv"), "-b", "4"])
    df = pd.read_csv(out)
    assert list(df.columns) == meta["columns"]
    assert list(df["data_ix"].to_numpy()[:16]) == list(z["row_order"])
    probs = np.zeros_like(z["probs"])
    probs[df["data_ix"].to_numpy(), df["category_ix"].to_numpy().astype(int)] = df["prob"].to_numpy()
    assert np.abs(probs - z["probs"]).max() <= 1e-5
    assert (probs.argmax(1) == z["argmax"]).all()


@pytest.mark.parametrize("ref_csv,flags", [("ref_plain_encode.csv", ["-b", "3"]),
                                           ("ref_plain_encode_named.csv", ["-b", "4", "-p", "mean,log_variance"])])
def test_reference_plain_checkpoint_encodes_like_reference(tmp_path, ref_csv, flags):
    """plain/encode.py:12-61 drop-in: a plain-VAE checkpoint WRITTEN BY THE
    REFERENCE CLI (tests/golden/ref_ckpt_plain.pt, make_golden.py:run_ckpt_plain)
    is opened through plain_learning.Learner.retrieve_model and plain_encode.py
    writes the reference's table: identical columns and column order, identical
    (data_ix, parameter_name, feature_dim) rows in the same order, identical
    annotation columns (speaker mapped as plain/modules/data_utils.py:17-22),
    parameter values (encoder + plain Sampler MLP kernels) <= 1e-5."""
    import numpy as np
    import plain_encode
    ref = pd.read_csv(os.path.join(GOLDEN, ref_csv))
    out = plain_encode.main([os.path.join(GOLDEN, "ref_ckpt_plain.pt"), TOY, ANN, "1.0", "-S",
                             os.path.join(str(tmp_path), "enc.csv")] + flags)
    got = pd.read_csv(out)
    assert list(got.columns) == list(ref.columns)
    assert len(got) == len(ref)
    for c in ref.columns:
        if c == "parameter_value":
            continue
        assert got[c].astype(str).tolist() == ref[c].astype(str).tolist(), c
    err = np.abs(got["parameter_value"].to_numpy() - ref["parameter_value"].to_numpy()).max()
    assert err <= 1e-5, err


def test_toy_trajectory_gpu_featurize_matches_reference(tmp_path):
    """The reference CLI's lstm_softmax_e2 trajectory with the STFT + log +
    packing on the GPU (--gpu_featurize, DeviceFeaturizer) instead of the host
    torch.stft chain: every logged training batch loss and the epoch totals
    within 1e-4 of the reference run (data_utils.py:88-103, 124-139, 165-182)."""
    ka = known_answers()["lstm_softmax_e2"]
    learner, _ = _run(tmp_path, ka["flags"] + ["--gpu_featurize"], "gpufeat")
    hist = learner.history
    for e in range(2):
        assert _rel(hist[e]["train"]["total"], ka["train_total"][e]) < 1e-4, (e, hist[e]["train"], ka)
        assert _rel(hist[e]["valid"]["total"], ka["valid_total"][e]) < 1e-4, (e, hist[e]["valid"], ka)
    losses = [x for e in range(2) for x in hist[e]["train"]["batch_loss"]]
    assert len(losses) == len(ka["batch_loss"])
    for a, b in zip(losses, ka["batch_loss"]):
        assert _rel(a, b) < 1e-4
