"""GPU featurisation + packing (abcd_featurize_packed) against the host path.

The reference's data path per item is Dataset.__getitem__ -> STFT ->
log_and_normalize, then pack_sequence (data_utils.py:88-103, 124-139,
165-182; learning.py:456-466); modules/data_utils.py restates it on the CPU
(torch.stft).  Here DeviceFeaturizer / DataLoader(featurizer=...) must give
the same batch order, batch_sizes and is_offset exactly.  Log-amplitudes:
the GPU evaluates each bin's DFT in fp64 (exact products of the fp32 samples
and the fp32 window), so it is held to a float64 torch.stft ground truth on
the same window values within 1e-5 -- no looser than the reference's own
fp32 host path; inputs are unscaled int16-valued samples, as the reference
feeds them.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _host_features(waves, n_fft, hop, center, eps, norm):
    from modules import data_utils as du
    stft = du.STFT(n_fft, hop, centering=center)
    feats = [(stft(torch.from_numpy(w)) + eps).log() / norm for w in waves]
    offs = [torch.tensor([0.0] * (f.shape[0] - 1) + [1.0]) for f in feats]
    return torch.nn.utils.rnn.pack_sequence(feats), torch.nn.utils.rnn.pack_sequence(offs)


@pytest.mark.parametrize("n_fft,hop,center", [(128, 64, True), (256, 128, True), (128, 64, False), (100, 33, True)])
def test_featurizer_matches_host_stft(n_fft, hop, center):
    from modules import data_utils as du
    g = np.random.default_rng(5)
    lens = sorted((int(x) for x in g.integers(n_fft, 40 * hop, size=37)), reverse=True)
    waves = [np.round(g.normal(0, 3000, size=n)).astype(np.float32) for n in lens]
    eps, norm = 2 ** (-15), 1.7
    ref, ref_off = _host_features(waves, n_fft, hop, center, eps, norm)
    fz = du.DeviceFeaturizer(n_fft, hop, centering=center, eps=eps, normalizer=norm, device="cuda")
    data, bs, is_off = fz(waves)
    torch.cuda.synchronize()
    assert torch.equal(bs, ref.batch_sizes)
    assert torch.equal(is_off.cpu(), ref_off.data)
    win = torch.hann_window(n_fft).double()  # the fp32 window both paths use, exactly
    truth = torch.nn.utils.rnn.pack_sequence([
        (torch.stft(torch.from_numpy(w).double(), n_fft, hop_length=hop, window=win, center=center,
                    return_complex=True).abs().T + eps).log() / norm for w in waves]).data
    gpu_err = (data.cpu().double() - truth).abs().max().item()
    host_err = (ref.data.double() - truth).abs().max().item()
    assert gpu_err <= max(1e-5, host_err), (gpu_err, host_err)


def test_dataloader_featurizer_batches(tmp_path):
    """A CSV + WAV dataset through DataLoader(featurizer=...): same batches
    (order, members, speakers) as the host path, features within 1e-4."""
    import scipy.io.wavfile as spw
    from modules import data_utils as du
    fs = 16000
    g = np.random.default_rng(11)
    rows = []
    for k in range(3):
        x = np.round(g.normal(0, 2000, size=fs)).astype(np.int16)
        spw.write(str(tmp_path / f"a{k}.wav"), fs, x)
        for j in range(4):
            on = float(g.uniform(0, 0.5))
            rows.append(f"a{k}.wav,{on:.4f},{on + float(g.uniform(0.05, 0.4)):.4f},s{j % 2},train")
    csv = tmp_path / "ann.csv"
    csv.write_text("input_path,onset,offset,speaker,data_type\n" + "\n".join(rows) + "\n")
    n_fft, hop, eps, norm = 128, 64, 2 ** (-15), 1.0
    parser = du.Data_Parser(str(tmp_path), str(csv))
    host_ds = parser.get_data(data_type="train", transform=du.Compose([
        du.ToTensor(), du.STFT(n_fft, hop), du.Transform(lambda x: (x + eps).log() / norm)]))
    raw_ds = parser.get_data(data_type="train", transform=None)
    torch.manual_seed(3)
    host = [(p.data.clone(), p.batch_sizes.clone(), o.data.clone(), list(ix))
            for p, o, _, ix in du.DataLoader(host_ds, batch_size=5, shuffle=True)]
    torch.manual_seed(3)
    fz = du.DeviceFeaturizer(n_fft, hop, eps=eps, normalizer=norm)
    dev = [(p.data.cpu(), p.batch_sizes.clone(), o.data.cpu(), list(ix))
           for p, o, _, ix in du.DataLoader(raw_ds, batch_size=5, shuffle=True, featurizer=fz)]
    assert len(host) == len(dev)
    for (hd, hb, ho, hix), (dd, db, do, dix) in zip(host, dev):
        assert hix == dix
        assert torch.equal(hb, db)
        assert torch.equal(ho, do)
        assert (hd - dd).abs().max().item() < 1e-3


def test_featurizer_matches_reference_toy_batch():
    """Pinned to the REFERENCE pipeline's own output: the first toy training
    batch as the reference's data_utils built it (Data_Parser -> STFT ->
    log_and_normalize -> DataLoader pop-from-end -> pack_sequence;
    tests/golden/toy_step.npz, make_golden.py:run_toy_step) against
    DeviceFeaturizer on the same segments' raw samples: identical
    batch_sizes and is_offset; log-amplitudes as close to the reference's as
    the reference's own fp32 STFT is to the float64 truth (elementwise, + 1e-5:
    near-empty bins amplify the fp32 rounding of |X| through the log), and no
    further from that truth than the reference (or 1e-5)."""
    from modules import data_utils as du
    from golden_io import GOLDEN
    z = np.load(os.path.join(GOLDEN, "toy_step.npz"), allow_pickle=False)
    toy = os.path.join(GOLDEN, "toy_data")
    parser = du.Data_Parser(toy, os.path.join(toy, "annotation_20170806-080002_89.2-94.22.csv"))
    fs = parser.get_sample_freq()
    frame, hop = int(np.floor(0.008 * fs)), int(np.floor(0.004 * fs))
    raw = parser.get_data(data_type="train", transform=None)
    ixs = [int(i) for i in z["ixs"]]  # annotation labels, already in the batch's packed (length-descending) order
    waves = [raw[ix][0] for ix in ixs]
    fz = du.DeviceFeaturizer(frame, hop, eps=2 ** (-15), normalizer=1.0, device="cuda")
    data, bs, is_off = fz(waves)
    torch.cuda.synchronize()
    assert torch.equal(bs, torch.from_numpy(z["batch_sizes"]))
    assert torch.equal(is_off.cpu(), torch.from_numpy(z["is_offset"]))
    win = torch.hann_window(frame).double()
    truth = torch.nn.utils.rnn.pack_sequence([
        (torch.stft(torch.from_numpy(w).double(), frame, hop_length=hop, window=win, center=True,
                    return_complex=True).abs().T + 2 ** (-15)).log() for w in waves]).data
    ref = torch.from_numpy(z["data"]).double()
    got = data.cpu().double()
    gpu_err, ref_err = (got - truth).abs().max().item(), (ref - truth).abs().max().item()
    assert gpu_err <= max(1e-5, ref_err), (gpu_err, ref_err)
    slack = (ref - truth).abs() + 1e-5
    assert bool(((got - ref).abs() <= slack).all()), float(((got - ref).abs() - slack).max())
