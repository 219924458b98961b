# coding: utf-8
"""Post-training encoding (ABCD-VAE/encode.py): encoder -> sampler logits ->
softmax -> long-format CSV (data_ix, category_ix, prob, annotation columns).
Runs the encoder and sampler forward on the HIP path."""
import argparse
import os

import numpy as np
import pandas as pd
import torch

import learning
from modules import data_utils
from modules.data_utils import Compose

OUTPUT = "probs"  # encode_logit.py -> "logits", encode_features.py -> "features"


class Encoder(learning.Learner):
    """encode.py:12-55"""

    def __init__(self, model_config_path, device="cuda"):
        self.device = torch.device(device)
        self.retrieve_model(checkpoint_path=model_config_path, device=device)
        for param in self.parameters():
            param.requires_grad = False
        self.encoder.eval()
        self.feature_sampler.eval()
        self.decoder.eval()

    def encode(self, data, is_packed=False, to_numpy=True, output=None):
        output = output or OUTPUT
        if not is_packed:
            if not isinstance(data, list):
                data = [data]
            data = torch.nn.utils.rnn.pack_sequence(data)
        with torch.no_grad():
            data = data.to(self.device)
            last_hidden = self.encoder(data)
            if output == "features":
                out = self.feature_sampler.to_code_like(last_hidden)
            else:
                out = self.feature_sampler(last_hidden)
                if output == "probs":
                    out = torch.nn.functional.softmax(out, -1)
        if to_numpy:
            out = (p.data.cpu().numpy() for p in out)
        return out

    def encode_dataset(self, dataset, save_path, to_numpy=True, batch_size=1, output=None):
        output = output or OUTPUT
        var_name, value_name = {"probs": ("category_ix", "prob"), "logits": ("dimension", "logit"),
                                "features": ("dimension", "feature_value")}[output]
        dataloader = data_utils.DataLoader(dataset, batch_size=batch_size)
        rename_existing_file(save_path)
        if "label" in dataset.df_annotation.columns:
            df_ann = dataset.df_annotation.drop(columns=["onset_ix", "offset_ix", "length"])
        else:
            df_ann = None
        for data, _, _, ix_in_list in dataloader:
            vals = self.encode(data, is_packed=True, to_numpy=to_numpy, output=output)
            df_encoded = pd.DataFrame(vals)
            df_encoded.loc[:, "data_ix"] = ix_in_list
            df_encoded = df_encoded.melt(id_vars=["data_ix"], var_name=var_name, value_name=value_name)
            if df_ann is not None:
                df_encoded = df_encoded.merge(df_ann, how="left", left_on="data_ix", right_index=True)
            if os.path.isfile(save_path):
                df_encoded.to_csv(save_path, index=False, mode="a", header=False)
            else:
                df_encoded.to_csv(save_path, index=False)


def rename_existing_file(filepath):
    if os.path.isfile(filepath):
        new_path = filepath + ".prev"
        rename_existing_file(new_path)
        os.rename(filepath, new_path)


def get_parameters(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("model_path", type=str, help="Path to the configuration file of a trained model.")
    p.add_argument("input_root", type=str, help="Path to the root directory under which inputs are located.")
    p.add_argument("annotation_file", type=str, help="Path to the annotation csv file.")
    p.add_argument("data_normalizer", type=float, help="Normalizing constant to devide the data.")
    p.add_argument("--annotation_sep", type=str, default=",", help="Separator symbol of the annotation file.")
    p.add_argument("-d", "--device", type=str, default="cuda", help="Computing device (GPU only).")
    p.add_argument("-S", "--save_path", type=str, default=None, help="Path to the file where results are saved.")
    p.add_argument("--fft_frame_length", type=float, default=0.008, help="FFT frame length in sec.")
    p.add_argument("--fft_step_size", type=float, default=0.004, help="FFT step size in sec.")
    p.add_argument("--fft_window_type", type=str, default="hann_window", help="Window type for FFT.")
    p.add_argument("--fft_no_centering", action="store_true", help="If selected, no centering in FFT.")
    p.add_argument("--channel", type=int, default=0, help="Channel ID # of multichannel recordings to use.")
    p.add_argument("-E", "--epsilon", type=float, default=2 ** (-15), help="Added before log.")
    p.add_argument("-b", "--batch_size", type=int, default=1, help="Batch size.")
    return p.parse_args(argv)


def main(argv=None, output=None):
    parameters = get_parameters(argv)
    save_path = parameters.save_path
    if save_path is None:
        save_path = os.path.join(parameters.input_root, "autoencoded.csv")
    save_dir = os.path.dirname(save_path)
    if save_dir and not os.path.isdir(save_dir):
        os.makedirs(save_dir)
    data_parser = data_utils.Data_Parser(parameters.input_root, parameters.annotation_file,
                                         annotation_sep=parameters.annotation_sep)
    fs = data_parser.get_sample_freq()
    fft_frame_length = int(np.floor(parameters.fft_frame_length * fs))
    fft_step_size = int(np.floor(parameters.fft_step_size * fs))
    encoder = Encoder(parameters.model_path, device=parameters.device)
    to_tensor = data_utils.ToTensor()
    stft = data_utils.STFT(fft_frame_length, fft_step_size, window=parameters.fft_window_type,
                           centering=not parameters.fft_no_centering)
    eps, norm = parameters.epsilon, parameters.data_normalizer
    log_and_normalize = data_utils.Transform(lambda x: (x + eps).log() / norm)
    dataset = data_parser.get_data(transform=Compose([to_tensor, stft, log_and_normalize]),
                                   channel=parameters.channel)
    encoder.encode_dataset(dataset, save_path, batch_size=parameters.batch_size, output=output)
    return save_path


if __name__ == "__main__":
    main()
