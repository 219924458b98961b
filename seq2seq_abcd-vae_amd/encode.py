# coding: utf-8
"""Post-training encoding on the HIP path: the drop-in for ABCD-VAE/encode.py
(and, through ``output=``, encode_logit.py / encode_features.py).

Same command line and the same long-format CSV as the reference
(encode.py:38-55): one row per (segment, category) with columns
``data_ix, category_ix, prob`` (``dimension, logit`` / ``dimension,
feature_value`` for the logit / feature variants) followed by the
annotation columns, rows ordered category-major within each batch.

How it runs here: every batch goes through the encoder and sampler forward
kernels once (model.py:60-66, 581-590) and stays on the device; the softmax
(or nothing, or the to_code_like MLP) is applied there, and the table is
written batch by batch with numpy index arithmetic (no DataFrame melt /
merge / append cycle), the previous batch's rows while the current one runs."""
import argparse
import os

import numpy as np
import pandas as pd
import torch

import learning
from modules import _native, data_utils
from modules.data_utils import Compose

OUTPUT = "probs"  # encode_logit.py -> "logits", encode_features.py -> "features"
COLUMNS = {"probs": ("category_ix", "prob"), "logits": ("dimension", "logit"),
           "features": ("dimension", "feature_value")}


class Encoder(learning.Learner):
    """A trained checkpoint (ours or the reference's: learning.py:317-347 keys)
    opened for inference: parameters frozen, modules in eval mode."""

    def __init__(self, model_config_path, device="cuda"):
        self.device = torch.device(device)
        self.retrieve_model(checkpoint_path=model_config_path, device=device)
        for m in (self.encoder, self.feature_sampler, self.decoder):
            m.requires_grad_(False)
            m.eval()

    def _device_output(self, packed, output):
        with torch.no_grad():
            h = self.encoder(packed.to(self.device))
            if output == "features":
                return self.feature_sampler.to_code_like(h)
            logits = self.feature_sampler(h)
            return torch.softmax(logits, -1) if output == "probs" else logits

    def encode(self, data, is_packed=False, to_numpy=True, output=None):
        """One batch (a PackedSequence, a tensor or a list of tensors) ->
        B x K probabilities (or logits / features); with to_numpy, an iterator
        of per-segment numpy rows as the reference returns."""
        if not is_packed:
            data = torch.nn.utils.rnn.pack_sequence(data if isinstance(data, list) else [data])
        out = self._device_output(data, output or OUTPUT)
        if to_numpy:
            return iter(out.cpu().numpy())
        return out

    def encode_dataset(self, dataset, save_path, to_numpy=True, batch_size=1, output=None):
        """Streams the table: each batch's device output is copied to pinned
        host memory without blocking, and the PREVIOUS batch's rows are written
        while the current one computes, so host and device memory stay bounded
        by two batches whatever the dataset size (the reference also writes
        per batch, encode.py:38-55)."""
        output = output or OUTPUT
        var_name, value_name = COLUMNS[output]
        # the table is written to a temporary path and takes save_path (the
        # earlier output kept as .prev) only once every batch is written and
        # the device status is clean: a timed-out persistent launch or an error
        # part way leaves no invalid or partial table behind
        tmp_path = save_path + ".partial"
        ann = None
        if "label" in dataset.df_annotation.columns:
            ann = dataset.df_annotation.drop(columns=["onset_ix", "offset_ix", "length"])
        state = {"header": True}

        def write(host, event, ix):
            event.synchronize()
            v = host.numpy()
            n, k = v.shape
            table = pd.DataFrame({"data_ix": np.tile(ix, k), var_name: np.repeat(np.arange(k), n),
                                  value_name: v.T.reshape(-1)})
            if ann is not None:
                extra = ann.reindex(table["data_ix"].to_numpy()).reset_index(drop=True)
                table = pd.concat([table, extra], axis=1)
            table.to_csv(tmp_path, index=False, mode="w" if state["header"] else "a", header=state["header"])
            state["header"] = False

        try:
            pending = None
            for packed, _, _, ix in data_utils.DataLoader(dataset, batch_size=batch_size):
                vals = self._device_output(packed, output)
                host = torch.empty(vals.shape, dtype=vals.dtype, pin_memory=True)
                host.copy_(vals, non_blocking=True)
                event = torch.cuda.Event()
                event.record()
                if pending is not None:
                    write(*pending)
                pending = (host, event, np.asarray(ix, dtype=np.int64))
            if pending is not None:
                write(*pending)
            _native.op_status.sync("encode_dataset")  # a timed-out persistent launch fails the run, not the table
        except BaseException:
            if os.path.isfile(tmp_path):
                os.remove(tmp_path)
            raise
        if os.path.isfile(tmp_path):  # (an empty dataset writes no table, as the reference)
            rename_existing_file(save_path)
            os.replace(tmp_path, save_path)


def rename_existing_file(filepath):
    """Keep earlier outputs: path -> path.prev -> path.prev.prev -> ..."""
    chain = []
    p = filepath
    while os.path.isfile(p):
        chain.append(p)
        p += ".prev"
    for src in reversed(chain):
        os.rename(src, src + ".prev")


def get_parameters(argv=None):
    p = argparse.ArgumentParser(description="Encode annotated segments with a trained ABCD-VAE (MI355X).")
    p.add_argument("model_path", type=str, help="checkpoint.pt written by learning.py (this package or the reference)")
    p.add_argument("input_root", type=str, help="directory the annotation's wav paths are relative to")
    p.add_argument("annotation_file", type=str, help="annotation table (csv) of the segments to encode")
    p.add_argument("data_normalizer", type=float, help="log-amplitudes are divided by this (training's -N)")
    p.add_argument("--annotation_sep", type=str, default=",", help="field separator of the annotation table")
    p.add_argument("-d", "--device", type=str, default="cuda", help="GPU device (there is no CPU path)")
    p.add_argument("-S", "--save_path", type=str, default=None,
                   help="output csv (default: <input_root>/autoencoded.csv); an existing file is kept as .prev")
    p.add_argument("--fft_frame_length", type=float, default=0.008, help="STFT window length, seconds")
    p.add_argument("--fft_step_size", type=float, default=0.004, help="STFT hop, seconds")
    p.add_argument("--fft_window_type", type=str, default="hann_window", help="torch window function name")
    p.add_argument("--fft_no_centering", action="store_true", help="STFT without centre padding")
    p.add_argument("--channel", type=int, default=0, help="channel (0-based) of multi-channel wav files")
    p.add_argument("-E", "--epsilon", type=float, default=2 ** (-15), help="offset inside log(|STFT| + eps)")
    p.add_argument("-b", "--batch_size", type=int, default=1, help="segments per forward pass")
    return p.parse_args(argv)


def main(argv=None, output=None):
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
    enc.encode_dataset(parser.get_data(transform=tfm, channel=a.channel), save_path, batch_size=a.batch_size,
                       output=output)
    return save_path


if __name__ == "__main__":
    main()
