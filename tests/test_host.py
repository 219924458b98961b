"""CPU-side tests of the product package: the C-ABI library loads and exports
every symbol include/abcd_hip.h declares (no compute without a GPU), the
nn.Module surface has the reference's names / init / state_dict, and compute
refuses CPU tensors (no silent fallback)."""
import hashlib
import os
import re

import pytest
import torch

from golden_io import SMALL, load_small, params_from, load_toy
from gpu_helpers import build_from_meta

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "abcd_hip.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(abcd_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_header_symbols():
    from modules import _native as N
    lib = N.lib()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert set(N.EXPORTED) == set(syms), set(N.EXPORTED) ^ set(syms)
    assert b"gfx950" in lib.abcd_version()
    from modules import _native
    assert _native.library_hash() == _native.source_hash()  # the loaded library is this tree's build


def test_workspace_queries_without_gpu():
    from modules import _native as N
    c = N.EncoderCfg(129, 256, N.LSTM, 1, 1)
    assert N.lib().abcd_encoder_out_size(c) == 1024
    assert N.lib().abcd_encoder_workspace_bytes(c, 200, 65583, 512) > 65583 * 256 * 4
    bad = N.EncoderCfg(129, 250, N.LSTM, 1, 1)
    assert N.lib().abcd_encoder_workspace_bytes(bad, 200, 65583, 512) == 0


@pytest.mark.parametrize("name", SMALL)
def test_init_and_state_dict_match_reference(name):
    meta, arr = load_small(name)
    enc, samp, dec = build_from_meta(meta, None, device="cpu")
    ref = params_from(arr)
    ours = {}
    for pfx, m in (("encoder", enc), ("feature_sampler", samp), ("decoder", dec)):
        ours.update({f"{pfx}/{k}": v for k, v in m.state_dict().items()})
    assert list(ours) == list(ref)
    for k in ref:
        assert torch.equal(ours[k], ref[k]), k


def test_toy_init_checksums():
    from modules import model as M
    cks, toy = load_toy()
    torch.manual_seed(1111)
    enc = M.RNN_Variational_Encoder(65, 256, rnn_type="LSTM")
    samp = M.ABCDSampler(enc.hidden_size_total, 256, 16, 256)
    dec = M.RNN_Variational_Decoder(65, 256, 256, 256, rnn_type="LSTM")
    for name, m in (("encoder", enc), ("feature_sampler", samp), ("decoder", dec)):
        h = hashlib.sha256()
        for v in m.state_dict().values():
            h.update(v.detach().contiguous().numpy().tobytes())
        assert h.hexdigest()[:16] == cks[name][1], name


def test_pack_init_parameters_roundtrip():
    from modules import model as M
    enc = M.RNN_Variational_Encoder(65, 32, rnn_type="GRU", rnn_layers=2)
    p = enc.pack_init_parameters()
    assert p == {"input_size": 65, "rnn_hidden_size": 32, "rnn_type": "GRU", "rnn_layers": 2,
                 "hidden_dropout": 0.0, "bidirectional": True}
    enc2 = M.RNN_Variational_Encoder(**p)
    enc2.load_state_dict(enc.state_dict())
    samp = M.ABCDSampler(enc.hidden_size_total, 32, 16, 32)
    s2 = M.ABCDSampler(**samp.pack_init_parameters())
    s2.load_state_dict(samp.state_dict())
    dec = M.RNN_Variational_Decoder(65, 32, 32, 32, num_speakers=3, speaker_embed_dim=16)
    d2 = M.RNN_Variational_Decoder(**dec.pack_init_parameters())
    d2.load_state_dict(dec.state_dict())


def test_temperature_schedule():
    """tau = min(min_temperature, exp(-rate * steps)), refreshed every 1000
    iterations: min_temperature acts as a cap (model.py:644-658)."""
    import math
    from modules import model as M
    s = M.ABCDSampler(32, 32, 16, 32)
    assert s.temperature == 1.0
    for _ in range(999):
        s.increment_iter_counts()
    assert s.temperature == 1.0
    s.increment_iter_counts()
    assert s.temperature == math.exp(-1e-5 * 1000)
    s2 = M.ABCDSampler(32, 32, 16, 32, min_temperature=0.5)
    assert s2.temperature == 0.5
    s3 = M.ABCDSampler(32, 32, 16, 32, epoch_init_iter_counts=2500)
    assert s3.temperature == math.exp(-1e-5 * 2000)


def test_compute_refuses_cpu_tensors():
    from modules import model as M
    enc = M.RNN_Variational_Encoder(33, 32)
    x = torch.nn.utils.rnn.pack_sequence([torch.randn(5, 33), torch.randn(3, 33)])
    with pytest.raises(RuntimeError):
        enc(x)


@pytest.mark.parametrize("n_fft,hop,center", [(128, 64, True), (256, 128, True), (128, 64, False), (100, 33, True)])
def test_stft_frame_count_matches_torch(n_fft, hop, center):
    """abcd_stft_frames (host function of the C ABI, no GPU) agrees with
    torch.stft's frame count -- the featuriser's batch_sizes depend on it."""
    from modules import _native as N
    lib = N.lib()
    for length in (n_fft // 2 + 1, n_fft, n_fft + 1, 1000, 4097):
        if not center and length < n_fft:
            continue
        z = torch.stft(torch.zeros(length), n_fft, hop_length=hop, window=torch.hann_window(n_fft), center=center,
                       return_complex=True)
        assert lib.abcd_stft_frames(length, n_fft, hop, int(center)) == z.shape[1], length


def test_reference_checkpoint_loads_into_product_modules():
    """A checkpoint written by the reference CLI loads with a loader that
    executes nothing (weights_only=True), and its *_init_parameters dicts and
    state dicts rebuild the product's modules exactly (learning.py:317-327)."""
    from modules import model as M
    path = os.path.join(REPO, "tests", "golden", "ref_ckpt_small.pt")
    ck = torch.load(path, map_location="cpu", weights_only=True)
    for k in ("epoch", "encoder", "encoder_init_parameters", "feature_sampler", "feature_sampler_init_parameters",
              "decoder", "decoder_init_parameters", "optimizer", "lr_scheduler", "gradient_clip", "random_state"):
        assert k in ck, k
    enc = M.RNN_Variational_Encoder(**ck["encoder_init_parameters"])
    samp = M.ABCDSampler(**ck["feature_sampler_init_parameters"])
    dec = M.RNN_Variational_Decoder(**ck["decoder_init_parameters"])
    for m, key in ((enc, "encoder"), (samp, "feature_sampler"), (dec, "decoder")):
        m.load_state_dict(ck[key])
        for name, v in m.state_dict().items():
            assert torch.equal(v, ck[key][name]), (key, name)


def test_custom_ops_registered():
    """The module classes call the C ABI through torch.library custom
    operators (modules/ops.py): every forward op has an autograd formula and a
    fake (meta) implementation, and takes no Python objects."""
    import torch
    from modules import ops
    assert list(ops.registered()) == list(ops.OPS)
    for name in ops.OPS:
        schema = str(getattr(torch.ops.abcd, name).default._schema)
        assert schema.startswith(f"abcd::{name}("), schema
        assert "(a!)" not in schema and "(a1!)" not in schema, schema  # functional: no mutated inputs
    assert ops._u64(ops._i64(0xF00DF00DF00DF00D)) == 0xF00DF00DF00DF00D


def test_reference_plain_checkpoint_oracle_encode():
    """The plain-VAE checkpoint written by the reference CLI
    (tests/golden/ref_ckpt_plain.pt) loads with weights_only=True into the
    product's plain modules, and the oracle's encoder + plain sampler
    (oracle/abcd_oracle.py: encoder_forward, plain_params) on the host data
    pipeline reproduce the reference plain/encode.py table
    (tests/golden/ref_plain_encode.csv) to <= 1e-5: this pins the checker the
    GPU test of plain_encode.py stands beside."""
    import numpy as np
    import pandas as pd
    from modules import data_utils, model as M
    from modules.data_utils import Compose
    from oracle import abcd_oracle as O
    g = os.path.join(REPO, "tests", "golden")
    ck = torch.load(os.path.join(g, "ref_ckpt_plain.pt"), map_location="cpu", weights_only=True)
    enc = M.RNN_Variational_Encoder(**ck["encoder_init_parameters"])
    samp = M.Sampler(**ck["feature_sampler_init_parameters"])
    enc.load_state_dict(ck["encoder"], strict=False)
    samp.load_state_dict(ck["feature_sampler"])
    P = {f"encoder/{k}": v for k, v in ck["encoder"].items()}
    P.update({f"feature_sampler/{k}": v for k, v in ck["feature_sampler"].items()})
    ei = ck["encoder_init_parameters"]
    cfg = dict(bidirectional=ei.get("bidirectional", True), layers=ei.get("rnn_layers", 1),
               rnn=ei.get("rnn_type", "LSTM"))
    toy = os.path.join(g, "toy_data")
    parser = data_utils.Data_Parser(toy, os.path.join(toy, "annotation_20170806-080002_89.2-94.22.csv"))
    fs = parser.get_sample_freq()
    frame, hop = int(np.floor(0.008 * fs)), int(np.floor(0.004 * fs))
    tfm = Compose([data_utils.ToTensor(), data_utils.STFT(frame, hop),
                   data_utils.Transform(lambda x: (x + 2 ** (-15)).log() / 1.0)])
    ref = pd.read_csv(os.path.join(g, "ref_plain_encode.csv"))
    f = ck["feature_sampler_init_parameters"]["output_size"]
    want = {}
    for p in (0, 1):
        sub = ref[ref.parameter_name == p]
        want[p] = sub.pivot(index="data_ix", columns="feature_dim", values="parameter_value").to_numpy()
    got = {0: np.zeros_like(want[0]), 1: np.zeros_like(want[1])}
    with torch.no_grad():
        for packed, _, _, ix in data_utils.DataLoader(parser.get_data(transform=tfm), batch_size=3):
            h = O.encoder_forward(P, packed.data, packed.batch_sizes, cfg)
            mu, lv = O.plain_params(P, h)
            got[0][np.asarray(ix)] = mu.numpy()
            got[1][np.asarray(ix)] = lv.numpy()
    assert want[0].shape[1] == f
    for p in (0, 1):
        assert np.abs(got[p] - want[p]).max() <= 1e-5, p
