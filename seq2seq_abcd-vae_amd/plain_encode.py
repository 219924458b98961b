# coding: utf-8
"""Post-training encoding of the plain Gaussian VAE on the HIP path: the
drop-in for plain/encode.py.

Same command line and the same long-format CSV as the reference
(plain/encode.py:37-52, 56-107): one row per (segment, Gaussian parameter,
feature dimension) with columns ``data_ix, parameter_name, feature_dim,
parameter_value``, sorted by (data_ix, parameter_name, feature_dim), then the
annotation columns when the annotation has a ``label`` column.
``parameter_name`` is the parameter's index (0 = mean, 1 = log-variance of
``Sampler.forward``, plain/modules/model.py:545-550) unless ``-p`` names
them.

How it runs here: each batch goes through the encoder kernels and the
plain sampler's MLP kernels once (model.py:60-66; plain model.py:545-550) and
its (mean, log-variance) rows stay on the device until the dataset is done;
the table is then built with numpy index arithmetic from two N x f host
matrices instead of one Python tuple per value.  The reference sorts the
whole table before writing it, so nothing is written per batch here either."""
import argparse
import os

import numpy as np
import pandas as pd
import torch

import plain_learning
from modules import _native, data_utils
from modules.data_utils import Compose

COLUMNS = ["data_ix", "parameter_name", "feature_dim", "parameter_value"]


class Encoder(plain_learning.Learner):
    """A trained plain checkpoint (ours or the reference's, plain/learning.py
    keys) opened for inference: parameters frozen, modules in eval mode
    (plain/encode.py:12-20)."""

    def __init__(self, model_config_path, device="cuda"):
        self.device = torch.device(device)
        self.retrieve_model(checkpoint_path=model_config_path, device=device)
        for m in (self.encoder, self.feature_sampler, self.decoder):
            m.requires_grad_(False)
            m.eval()

    def _device_params(self, packed):
        with torch.no_grad():
            h = self.encoder(packed.to(self.device))
            return self.feature_sampler(h)

    def encode(self, data, is_packed=False, to_numpy=True):
        """One batch -> the sampler's parameters [mean (B x f), log-variance
        (B x f)]; with to_numpy a generator of numpy arrays, as the reference
        returns (plain/encode.py:23-34)."""
        if not is_packed:
            data = torch.nn.utils.rnn.pack_sequence(data if isinstance(data, list) else [data])
        params = self._device_params(data)
        if to_numpy:
            return (p.cpu().numpy() for p in params)
        return params

    def encode_dataset(self, dataset, to_numpy=True, parameter_ix2name=None, batch_size=1):
        """plain/encode.py:37-52: the long table over the whole dataset,
        UNSORTED in the reference's row order (batch, parameter, segment,
        dimension); main() sorts it as the reference does."""
        if parameter_ix2name is None:
            parameter_ix2name = {}
        outs, ixs = [], []
        for packed, _, _, ix in data_utils.DataLoader(dataset, batch_size=batch_size):
            outs.append(self._device_params(packed))  # device tensors; copied once at the end
            ixs.append(np.asarray(ix, dtype=np.int64))
        _native.op_status.sync("encode_dataset")  # a timed-out persistent launch fails the run, not the table
        frames = []
        for params, ix in zip(outs, ixs):
            for pix, p in enumerate(params):
                v = p.cpu().numpy()
                n, f = v.shape
                name = parameter_ix2name.get(pix, pix)
                frames.append(pd.DataFrame({"data_ix": np.repeat(ix, f), "parameter_name": [name] * (n * f),
                                            "feature_dim": np.tile(np.arange(f), n),
                                            "parameter_value": v.reshape(-1)}))
        if not frames:
            return pd.DataFrame(columns=COLUMNS)
        return pd.concat(frames, ignore_index=True)[COLUMNS]


def plain_annotation(annotation_file, sep=","):
    """The annotation table as plain/modules/data_utils.py:10-22 leaves it
    (speaker ids mapped to their first-appearance index, or a NaN speaker
    column when there is none): the columns the reference's output carries."""
    df = pd.read_csv(annotation_file, sep=sep)
    if "speaker" in df.columns:
        speaker2ix = {spk: ix for ix, spk in enumerate(df.speaker.unique())}
        df.loc[:, "speaker"] = df.speaker.map(speaker2ix)
    else:
        df["speaker"] = float("nan")
    return df


def get_parameters(argv=None):
    p = argparse.ArgumentParser(description="Encode annotated segments with a trained plain VAE (MI355X).")
    p.add_argument("model_path", type=str, help="checkpoint.pt written by plain_learning.py or plain/learning.py")
    p.add_argument("input_root", type=str, help="directory the annotation's wav paths are relative to")
    p.add_argument("annotation_file", type=str, help="annotation table (csv) of the segments to encode")
    p.add_argument("data_normalizer", type=float, help="log-amplitudes are divided by this (training's -N)")
    p.add_argument("--annotation_sep", type=str, default=",", help="field separator of the annotation table")
    p.add_argument("-d", "--device", type=str, default="cuda", help="GPU device (there is no CPU path)")
    p.add_argument("-S", "--save_path", type=str, default=None,
                   help="output csv (default: <input_root>/autoencoded.csv)")
    p.add_argument("--fft_frame_length", type=float, default=0.008, help="STFT window length, seconds")
    p.add_argument("--fft_step_size", type=float, default=0.004, help="STFT hop, seconds")
    p.add_argument("--fft_window_type", type=str, default="hann_window", help="torch window function name")
    p.add_argument("--fft_no_centering", action="store_true", help="STFT without centre padding")
    p.add_argument("--channel", type=int, default=0, help="channel (0-based) of multi-channel wav files")
    p.add_argument("-p", "--parameter_names", type=str, default=None, help="comma-separated parameter names")
    p.add_argument("-E", "--epsilon", type=float, default=2 ** (-15), help="offset inside log(|STFT| + eps)")
    p.add_argument("-b", "--batch_size", type=int, default=1, help="segments per forward pass")
    return p.parse_args(argv)


def main(argv=None):
    a = get_parameters(argv)
    save_path = a.save_path or os.path.join(a.input_root, "autoencoded.csv")
    if os.path.dirname(save_path):
        os.makedirs(os.path.dirname(save_path), exist_ok=True)
    parser = data_utils.Data_Parser(a.input_root, a.annotation_file, annotation_sep=a.annotation_sep)
    fs = parser.get_sample_freq()
    frame, hop = int(np.floor(a.fft_frame_length * fs)), int(np.floor(a.fft_step_size * fs))
    enc = Encoder(a.model_path, device=a.device)
    eps, norm = a.epsilon, a.data_normalizer
    tfm = Compose([data_utils.ToTensor(),
                   data_utils.STFT(frame, hop, window=a.fft_window_type, centering=not a.fft_no_centering),
                   data_utils.Transform(lambda x: (x + eps).log() / norm)])
    ix2name = {} if a.parameter_names is None else dict(enumerate(a.parameter_names.split(",")))
    df = enc.encode_dataset(parser.get_data(transform=tfm, channel=a.channel), parameter_ix2name=ix2name,
                            batch_size=a.batch_size)
    df = df.sort_values(["data_ix", "parameter_name", "feature_dim"])
    ann = plain_annotation(a.annotation_file, a.annotation_sep)
    if "label" in ann.columns:
        df = df.merge(ann, how="left", left_on="data_ix", right_index=True)
    df.to_csv(save_path, index=False)
    return save_path


if __name__ == "__main__":
    main()
