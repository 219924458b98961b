"""Loading helpers for the committed golden fixtures (tests/golden/)."""
import json
import os
from collections import OrderedDict

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SMALL = sorted(f[len("small_"):-len(".npz")] for f in os.listdir(GOLDEN) if f.startswith("small_"))


def load_small(name):
    z = np.load(os.path.join(GOLDEN, f"small_{name}.npz"), allow_pickle=False)
    meta = json.loads(bytes(z["meta"]).decode())
    arr = {k: torch.from_numpy(np.array(z[k])) for k in z.files if k != "meta"}
    return meta, arr


def small_cfg(meta):
    from oracle.abcd_oracle import default_cfg
    d = meta["dims"]
    speaker = meta.get("speaker", False)
    return default_cfg(F=d["F"], H=d["H"], Hdec=d["H"], Hm=d["Hm"], D=d["D"], K=d["K"],
                       rnn=meta["rnn"], layers=meta.get("layers", 1),
                       bidirectional=meta.get("bidirectional", True), greedy=meta.get("greedy", False),
                       plain=meta.get("plain", False), fplain=d["FPLAIN"],
                       num_speakers=d["NSPK"] if speaker else None, speaker_dim=d["S"] if speaker else None)


def params_from(arr, prefix="p/"):
    return OrderedDict((k[len(prefix):], v) for k, v in arr.items() if k.startswith(prefix))


def batch_from(arr):
    return dict(data=arr["data"], batch_sizes=arr["batch_sizes"], is_offset=arr["is_offset"],
                speakers=arr["speakers"].long())


def noise_from(meta, arr):
    feat = arr["feat_noise"]
    if not meta.get("plain") and meta.get("pretrain"):
        feat = None
    return dict(feat=feat, eps=arr["eps"], xmask=arr.get("xmask"))


PROD = sorted(f[len("prod_"):-len(".npz")] for f in os.listdir(GOLDEN) if f.startswith("prod_"))


def load_prod(name):
    z = np.load(os.path.join(GOLDEN, f"prod_{name}.npz"), allow_pickle=False)
    meta = json.loads(bytes(z["meta"]).decode())
    arr = {k: torch.from_numpy(np.array(z[k])) for k in z.files if k != "meta"}
    return meta, arr


def sha16(t):
    import hashlib
    return hashlib.sha256(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()[:16]


def prod_inputs(meta):
    """Inputs of a production-shape fixture, regenerated from its seeds with
    torch's CPU generator (same calls as tests/golden/make_golden.py:run_prod,
    which stored the sha256 of each so a regeneration that differs fails).

    Lengths U{tmin..tmax} (first forced to tmax), sorted desc; frames
    x ~ N(0,1); speakers U{0..nspk-1}; then, from a second generator, the
    step's noise in the reference's draw order: Gumbel -log(Exp(1)) (B x K)
    unless pretraining (plain: randn(B, f)), then randn(bs_t, F) per decoder
    step (model.py:604, 19)."""
    d = meta["dims"]
    F, B = d["F"], meta["B"]
    g = torch.Generator().manual_seed(meta["seed_data"])
    lens = torch.randint(meta["tmin"], meta["tmax"] + 1, (B,), generator=g)
    lens[0] = meta["tmax"]
    lens, _ = torch.sort(lens, descending=True)
    seqs = [torch.randn(int(T), F, generator=g) for T in lens]
    spk = torch.randint(0, max(d.get("NSPK") or 1, 1), (B,), generator=g)
    packed = torch.nn.utils.rnn.pack_sequence(seqs)
    is_off = torch.nn.utils.rnn.pack_sequence([torch.tensor([0.0] * (int(T) - 1) + [1.0]) for T in lens]).data
    gn = torch.Generator().manual_seed(meta["seed_noise"])
    if meta.get("plain"):
        feat_noise = torch.randn(B, d["FPLAIN"], generator=gn)
    elif not meta.get("pretrain", False):
        feat_noise = -torch.empty(B, d["K"]).exponential_(generator=gn).log()
    else:
        feat_noise = None
    eps = torch.cat([torch.randn(int(bs), F, generator=gn) for bs in packed.batch_sizes], 0)
    return dict(data=packed.data, batch_sizes=packed.batch_sizes, is_offset=is_off, speakers=spk,
                feat_noise=feat_noise, eps=eps, lengths=lens)


def known_answers():
    with open(os.path.join(GOLDEN, "toy_known_answers.json")) as f:
        return json.load(f)


def load_toy():
    z = np.load(os.path.join(GOLDEN, "toy_step.npz"), allow_pickle=False)
    out = {k: torch.from_numpy(np.array(z[k])) for k in z.files if k != "checksums"}
    return json.loads(bytes(z["checksums"]).decode()), out
