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


def known_answers():
    with open(os.path.join(GOLDEN, "toy_known_answers.json")) as f:
        return json.load(f)


def load_toy():
    z = np.load(os.path.join(GOLDEN, "toy_step.npz"), allow_pickle=False)
    out = {k: torch.from_numpy(np.array(z[k])) for k in z.files if k != "checksums"}
    return json.loads(bytes(z["checksums"]).decode()), out
