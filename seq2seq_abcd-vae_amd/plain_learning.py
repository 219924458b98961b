# coding: utf-8
"""Trainer for the plain Gaussian-VAE variant (plain/learning.py): same encoder
and decoder kernels, the feature sampler is ``Sampler(E, mlp, f)`` with a
reparameterised Gaussian and a KL to N(0, I) (plain/learning.py:90,146-159).
Config 4 of BASELINE.json uses it to isolate the LSTM kernels."""
import argparse
import itertools

import torch

import learning
from learning import logger
from modules import engine, model, noise, parallel


class Learner(learning.Learner):
    def __init__(self, input_size, encoder_rnn_hidden_size, decoder_rnn_hidden_size, mlp_hidden_size, feature_size,
                 save_dir, encoder_rnn_type="LSTM", decoder_rnn_type="LSTM", encoder_rnn_layers=1,
                 bidirectional_encoder=True, encoder_hidden_dropout=0.0, decoder_input_dropout=0.0, device="cuda",
                 seed=1111, decoder_self_feedback=True, num_speakers=None, speaker_embed_dim=None,
                 noise_mode="philox", **unused):
        learning._check_device(device)
        from modules import parallel
        self.rank, self.world = parallel.world()
        self.retrieval, self.log_file_path = learning.update_log_handler(save_dir)
        self.save_dir = save_dir
        self.device = torch.device(device)
        noise.set_mode(noise_mode)
        if self.retrieval:
            self.last_epoch = self.retrieve_model(device=device)
            return
        torch.manual_seed(seed)
        torch.cuda.manual_seed_all(seed)
        noise.manual_seed(seed, rank=self.rank)
        self.seed = seed
        self.encoder = model.RNN_Variational_Encoder(input_size, encoder_rnn_hidden_size, rnn_type=encoder_rnn_type,
                                                     rnn_layers=encoder_rnn_layers,
                                                     hidden_dropout=encoder_hidden_dropout,
                                                     bidirectional=bidirectional_encoder)
        self.feature_sampler = model.Sampler(self.encoder.hidden_size_total, mlp_hidden_size, feature_size)
        self.decoder = model.RNN_Variational_Decoder(input_size, decoder_rnn_hidden_size, mlp_hidden_size, feature_size,
                                                     rnn_type=decoder_rnn_type, input_dropout=decoder_input_dropout,
                                                     self_feedback=decoder_self_feedback, num_speakers=num_speakers,
                                                     speaker_embed_dim=speaker_embed_dim)
        logger.info("Data to be encoded into {f}-dim features.".format(f=feature_size))
        self._finish_modules()

    def retrieve_model(self, checkpoint_path=None, device="cuda"):
        import os
        self.device = torch.device(device)
        if checkpoint_path is None:
            checkpoint_path = os.path.join(self.save_dir, "checkpoint.pt")
        self.checkpoint = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        self.encoder = model.RNN_Variational_Encoder(**self.checkpoint["encoder_init_parameters"])
        self.feature_sampler = model.Sampler(**self.checkpoint["feature_sampler_init_parameters"])
        self.decoder = model.RNN_Variational_Decoder(**self.checkpoint["decoder_init_parameters"])
        self.encoder.load_state_dict(self.checkpoint["encoder"], strict=False)
        self.feature_sampler.load_state_dict(self.checkpoint["feature_sampler"])
        self.decoder.load_state_dict(self.checkpoint["decoder"])
        if not hasattr(self, "rank"):
            self.rank, self.world = parallel.world()
        self._finish_modules()
        self.gradient_clip = self.checkpoint["gradient_clip"]
        self.seed = int(self.checkpoint.get("seed", 1111))
        torch.set_rng_state(self.checkpoint["random_state"])
        if "abcd_noise_state" in self.checkpoint:
            noise.set_state(self.checkpoint["abcd_noise_state"], rank=self.rank)
        return self.checkpoint["epoch"]

    def train(self, dataloader, is_pretraining=False):
        mean = super().train(dataloader, is_pretraining=False)
        return mean

    def learn(self, train_dataset, valid_dataset, num_epochs, batch_size_train, batch_size_valid, learning_rate=0.1,
              momentum=0.9, gradient_clip=0.25, patience=0, **unused):
        return super().learn(train_dataset, valid_dataset, num_epochs, batch_size_train, batch_size_valid,
                             pretrain_epochs=0, learning_rate=learning_rate, momentum=momentum,
                             gradient_clip=gradient_clip, patience=patience)


def get_parameters(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("input_root", type=str)
    p.add_argument("annotation_file", type=str)
    p.add_argument("--annotation_sep", type=str, default=",")
    p.add_argument("-S", "--save_root", type=str, default=None)
    p.add_argument("-j", "--job_id", type=str, default="NO_JOB_ID")
    p.add_argument("-s", "--seed", type=int, default=1111)
    p.add_argument("-d", "--device", type=str, default="cuda")
    p.add_argument("-e", "--epochs", type=int, default=20)
    p.add_argument("-b", "--batch_size", type=int, default=512)
    p.add_argument("--validation_batch_size", type=int, default=None)
    p.add_argument("-l", "--learning_rate", type=float, default=1.0)
    p.add_argument("-M", "--momentum", type=float, default=0.0)
    p.add_argument("-c", "--clip", type=float, default=1.0)
    p.add_argument("-p", "--patience", type=int, default=0)
    p.add_argument("-R", "--encoder_rnn_type", type=str, default="LSTM")
    p.add_argument("--decoder_rnn_type", type=str, default=None)
    p.add_argument("-f", "--feature_size", type=int, default=16)
    p.add_argument("--encoder_rnn_layers", type=int, default=1)
    p.add_argument("--encoder_rnn_hidden_size", type=int, default=256)
    p.add_argument("--decoder_rnn_hidden_size", type=int, default=256)
    p.add_argument("--mlp_hidden_size", type=int, default=256)
    p.add_argument("--speaker_embed_dim", type=int, default=None)
    p.add_argument("--encoder_hidden_dropout", type=float, default=0.0)
    p.add_argument("--decoder_input_dropout", type=float, default=0.0)
    p.add_argument("--greedy_decoder", action="store_true")
    p.add_argument("--unidirectional_encoder", action="store_true")
    p.add_argument("--fft_frame_length", type=float, default=0.008)
    p.add_argument("--fft_step_size", type=float, default=0.004)
    p.add_argument("--fft_window_type", type=str, default="hann_window")
    p.add_argument("--fft_no_centering", action="store_true")
    p.add_argument("--channel", type=int, default=0)
    p.add_argument("-N", "--data_normalizer", type=float, default=1.0)
    p.add_argument("-E", "--epsilon", type=float, default=2 ** (-15))
    p.add_argument("--noise", type=str, default="philox", choices=["philox", "reference"])
    return p.parse_args(argv)


def main(argv=None):
    import json
    import os

    import numpy as np

    from modules import data_utils
    from modules.data_utils import Compose
    P = get_parameters(argv)
    save_root = P.save_root if P.save_root is not None else P.input_root
    save_dir = learning.get_save_dir(save_root, P.job_id)
    parser = data_utils.Data_Parser(P.input_root, P.annotation_file, annotation_sep=P.annotation_sep)
    fs = parser.get_sample_freq()
    frame, step = int(np.floor(P.fft_frame_length * fs)), int(np.floor(P.fft_step_size * fs))
    if P.decoder_rnn_type is None:
        P.decoder_rnn_type = P.encoder_rnn_type
    lrn = Learner(int(frame / 2 + 1), P.encoder_rnn_hidden_size, P.decoder_rnn_hidden_size, P.mlp_hidden_size,
                  P.feature_size, save_dir, encoder_rnn_type=P.encoder_rnn_type, decoder_rnn_type=P.decoder_rnn_type,
                  encoder_rnn_layers=P.encoder_rnn_layers, bidirectional_encoder=not P.unidirectional_encoder,
                  encoder_hidden_dropout=P.encoder_hidden_dropout, decoder_input_dropout=P.decoder_input_dropout,
                  device=P.device, seed=P.seed, decoder_self_feedback=not P.greedy_decoder,
                  num_speakers=parser.get_num_speakers(), speaker_embed_dim=P.speaker_embed_dim, noise_mode=P.noise)
    eps, norm = P.epsilon, P.data_normalizer
    tf = Compose([data_utils.ToTensor(), data_utils.STFT(frame, step, window=P.fft_window_type,
                                                         centering=not P.fft_no_centering),
                  data_utils.Transform(lambda x: (x + eps).log() / norm)])
    train = parser.get_data(data_type="train", transform=tf, channel=P.channel)
    valid = parser.get_data(data_type="valid", transform=tf, channel=P.channel)
    lrn.learn(train, valid, P.epochs, P.batch_size, P.validation_batch_size or P.batch_size,
              learning_rate=P.learning_rate, momentum=P.momentum, gradient_clip=P.clip, patience=P.patience)
    return lrn


if __name__ == "__main__":
    main()
