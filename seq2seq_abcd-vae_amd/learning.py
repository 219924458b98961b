# coding: utf-8
"""Trainer and CLI with the reference's surface (ABCD-VAE/learning.py), running
the training step on MI355X through the fused HIP step (modules/engine.py).

Same flags, same ``history.log`` lines, same ``checkpoint.pt`` keys, same
resume semantics and the same RNG consumption order as the reference.  What
changes is where the step runs:

* ``Learner.train`` calls ``FusedStep.step`` (encoder -> sampler -> KL ->
  decoder -> loss -> backward -> clip -> SGD as one sequence of HIP kernels, no
  autograd, no host synchronisation inside the epoch); per-batch loss and
  perplexity values stay on the GPU and are written to the log at the end of
  the epoch, with the reference's wording.
* noise: ``--noise philox`` (default) draws Gumbel/Gaussian noise in-kernel;
  ``--noise reference`` draws it on the host from torch's CPU generator in the
  reference's order, so a run reproduces a reference CPU run's random numbers.
* data parallelism: launched under ``torch.distributed.run`` (one rank per
  GPU), every rank trains on its length-balanced shard of each batch and the
  flat gradient buffer is averaged by one RCCL all-reduce per step.
"""
import argparse
import itertools
import json
import math
import os
from logging import DEBUG, FileHandler, Formatter, getLogger

import numpy as np
import torch
import torch.distributed as dist

from modules import data_utils, engine, model, noise, parallel
from modules.data_utils import Compose

logger = getLogger(__name__)


def update_log_handler(file_dir):
    """learning.py:12-32"""
    for h in logger.handlers[:]:
        logger.removeHandler(h)
    log_file_path = os.path.join(file_dir, "history.log")
    retrieval = os.path.isfile(log_file_path)
    handler = FileHandler(filename=log_file_path)
    handler.setLevel(DEBUG)
    handler.setFormatter(Formatter("{asctime} - {levelname} - {message}", style="{"))
    logger.setLevel(DEBUG)
    logger.addHandler(handler)
    if retrieval:
        logger.info("LEARNING RETRIEVED.")
    else:
        logger.info("Logger set up.")
        logger.info("PyTorch ver.: {ver}".format(ver=torch.__version__))
    return retrieval, log_file_path


def _check_device(device):
    if not str(device).startswith("cuda"):
        raise RuntimeError("this trainer runs the ABCD-VAE step on the GPU (MI355X HIP kernels); "
                           "use -d cuda (there is no CPU path)")


class Learner(object):
    status_every = 16  # steps between the non-blocking STATUS reads (engine.StatusWatch)

    def __init__(self, input_size, encoder_rnn_hidden_size, decoder_rnn_hidden_size, mlp_hidden_size,
                 num_feature_categories, feature_dim, save_dir, encoder_rnn_type="LSTM", decoder_rnn_type="LSTM",
                 encoder_rnn_layers=1, bidirectional_encoder=True, bidirectional_decoder=False,
                 right2left_decoder_weight=0.5, encoder_hidden_dropout=0.0, decoder_input_dropout=0.0,
                 device="cuda", seed=1111, emission_distribution="isotropic_gaussian", decoder_self_feedback=True,
                 esn_leak=1.0, num_speakers=None, speaker_embed_dim=None, prior_concentration=1.0,
                 noise_mode="philox"):
        _check_device(device)
        self.rank, self.world = parallel.world()
        self.retrieval, self.log_file_path = update_log_handler(save_dir)
        self.save_dir = save_dir
        self.device = torch.device(device)
        logger.info("Device: {device}".format(device=device))
        logger.info("HIP library: {v}".format(v=model.N.lib().abcd_version().decode()))
        if noise_mode == "reference" and self.world > 1:
            # the reference draws from ONE global CPU generator for the whole
            # batch; seeded alike, every rank would draw the same noise for its
            # own shard, which no single-device run draws
            raise ValueError("--noise reference reproduces a single-device reference run; "
                             "use --noise philox (per-rank keys) with data parallelism")
        noise.set_mode(noise_mode)
        logger.info("Noise source: {m}".format(m=noise_mode))
        self.step = None
        if self.retrieval:
            self.last_epoch = self.retrieve_model(device=device)
            logger.info("Model retrieved.")
        else:
            torch.manual_seed(seed)
            torch.cuda.manual_seed_all(seed)
            noise.manual_seed(seed, rank=self.rank)
            self.seed = seed
            if encoder_hidden_dropout > 0.0 and encoder_rnn_layers == 1:
                logger.warning("Non-zero dropout cannot be used for the single-layer encoder RNN "
                               "(because there is no non-top hidden layers).")
                logger.info("encoder_hidden_dropout reset from {do} to 0.0.".format(do=encoder_hidden_dropout))
                encoder_hidden_dropout = 0.0
            self.encoder = model.RNN_Variational_Encoder(input_size, encoder_rnn_hidden_size,
                                                         rnn_type=encoder_rnn_type, rnn_layers=encoder_rnn_layers,
                                                         hidden_dropout=encoder_hidden_dropout,
                                                         bidirectional=bidirectional_encoder, esn_leak=esn_leak)
            self.feature_sampler = model.ABCDSampler(self.encoder.hidden_size_total, mlp_hidden_size,
                                                     num_feature_categories, feature_dim,
                                                     prior_concentration=prior_concentration)
            self.decoder = model.RNN_Variational_Decoder(
                input_size, decoder_rnn_hidden_size, mlp_hidden_size, feature_dim,
                emission_distr_name=emission_distribution, rnn_type=decoder_rnn_type,
                input_dropout=decoder_input_dropout, self_feedback=decoder_self_feedback, esn_leak=esn_leak,
                bidirectional=bidirectional_decoder, right2left_weight=right2left_decoder_weight,
                num_speakers=num_speakers, speaker_embed_dim=speaker_embed_dim)
            logger.info("Data are encoded into one of {num_cat} possible {feature_dim}-dim feature vectors.".format(
                num_cat=num_feature_categories, feature_dim=feature_dim))
            logger.info("Discrete categories are assumed to be distributed according to Categorical(pi), "
                        "with Dirichlet({}) prior on pi.".format(prior_concentration))
            logger.info("Conditioned on the RNN-transformed features, data are assumed to be distributed "
                        "according to {e}".format(e=emission_distribution))
            logger.info("Random seed: {seed}".format(seed=seed))
            logger.info("Type of RNN used for the encoder: {rnn_type}".format(rnn_type=encoder_rnn_type))
            logger.info("Type of RNN used for the decoder: {rnn_type}".format(rnn_type=decoder_rnn_type))
            logger.info("# of RNN hidden layers in the encoder RNN: {hl}".format(hl=encoder_rnn_layers))
            logger.info("# of hidden units in the encoder RNNs: {hs}".format(hs=encoder_rnn_hidden_size))
            logger.info("# of hidden units in the decoder RNNs: {hs}".format(hs=decoder_rnn_hidden_size))
            logger.info("# of hidden units in the MLPs: {hs}".format(hs=mlp_hidden_size))
            if bidirectional_encoder:
                logger.info("Encoder is bidirectional.")
            logger.info("Dropout rate in the non-top layers of the encoder RNN: {do}".format(
                do=encoder_hidden_dropout))
            logger.info("Self-feedback to the decoder: {f}".format(f=decoder_self_feedback))
            if decoder_self_feedback:
                logger.info("Dropout rate in the input to the decoder RNN: {do}".format(do=decoder_input_dropout))
            if speaker_embed_dim is not None:
                logger.info("Speaker ID # is embedded and fed to the decoder.")
                logger.info("# of speakers: {n}".format(n=num_speakers))
                logger.info("Embedding dimension: {d}".format(d=speaker_embed_dim))
            self._finish_modules()

    # ------------------------------------------------------------------ plumbing
    def _finish_modules(self):
        self.parameters = lambda: itertools.chain(self.encoder.parameters(), self.feature_sampler.parameters(),
                                                  self.decoder.parameters())
        self.encoder.to(self.device)
        self.feature_sampler.to(self.device)
        self.decoder.to(self.device)
        self.step = engine.FusedStep(self.encoder, self.feature_sampler, self.decoder, self.device)
        if self.world > 1:
            parallel.broadcast_parameters(self.step)
            parallel.attach(self.step)

    def _to_device(self, packed_input, is_offset, speaker):
        data = packed_input.data.to(self.device, non_blocking=True)
        return data, packed_input.batch_sizes, is_offset.data.to(self.device, non_blocking=True), \
            speaker.to(self.device, non_blocking=True)

    def _shard(self, packed_input, is_offset, speaker):
        """Rank's length-balanced shard of a global batch (parallel.shard_global_batch),
        or None when the global batch has fewer segments than ranks and this
        rank gets none (it still joins the all-reduce: FusedStep.empty_step)."""
        if self.world == 1:
            return packed_input, is_offset, speaker
        seqs = torch.nn.utils.rnn.unpack_sequence(packed_input)
        offs = torch.nn.utils.rnn.unpack_sequence(is_offset)
        mine = parallel.shard_global_batch([len(s) for s in seqs], self.rank, self.world)
        if not mine:
            return None
        return (torch.nn.utils.rnn.pack_sequence([seqs[i] for i in mine]),
                torch.nn.utils.rnn.pack_sequence([offs[i] for i in mine]), speaker[mine])

    def _momentum_views(self):
        if self.step.momentum_buf is None:
            return
        fl = self.step.flat
        for p, o in zip(fl.params, fl.offsets):
            self.optimizer.state[p]["momentum_buffer"] = self.step.momentum_buf[o:o + p.numel()].view_as(p)

    # ---------------------------------------------------------------- training
    def train(self, dataloader, is_pretraining=False):
        """learning.py:127-197"""
        self.encoder.train()
        self.feature_sampler.train()
        self.decoder.train()
        num_batches = dataloader.get_num_batches()
        num_strings = len(dataloader.dataset)
        records = []
        group = self.optimizer.param_groups[0]
        watch = engine.StatusWatch(self.device, every=self.status_every)
        for batch_ix, (packed_input, is_offset, speaker, _) in enumerate(dataloader, 1):
            # loss / batch_sizes[0] of the GLOBAL batch (learning.py:156) on every rank
            b_global = int(packed_input.batch_sizes[0])
            shard = self._shard(packed_input, is_offset, speaker)
            if shard is None:
                sc = self.step.empty_step(lr=group["lr"], momentum=group["momentum"], clip=self.gradient_clip)
            else:
                data, bsz, off, spk = self._to_device(*shard)
                sc = self.step.step(data, bsz, off, spk, num_strings, is_pretraining=is_pretraining, lr=group["lr"],
                                    momentum=group["momentum"], clip=self.gradient_clip, loss_batch=b_global)
            self._momentum_views()
            records.append(sc.clone())
            watch.update(records)
            if not is_pretraining and hasattr(self.feature_sampler, "increment_iter_counts"):
                self.feature_sampler.increment_iter_counts()
        watch.finish()
        recs = torch.stack(records)
        if self.world > 1:
            dist.all_reduce(recs, op=dist.ReduceOp.SUM)
            # LOSS sums to the global-batch loss; the perplexities are per-shard
            # diagnostics, averaged
            recs[:, engine.PPL_CLUSTER:engine.PPL_SHAPE + 1] /= self.world
        recs = recs.cpu()
        engine.check_status(recs, "training batch")
        recs = recs.double().numpy()
        for batch_ix, r in enumerate(recs, 1):
            logger.info("{batch_ix}/{num_batches} training batches complete. mean loss: {loss:5.4f}. Perplexity of "
                        "the posterior clustering probs.: {cluster_perplex:5.4f}. Perplexity of the mean clustering "
                        "probs. over minibatch: {batch_perplex:5.4f}. Perplexity of the posterior Dirichlet shape: "
                        "{shape_perplex:5.4f}".format(batch_ix=batch_ix, num_batches=num_batches,
                                                      loss=r[engine.LOSS], cluster_perplex=r[engine.PPL_CLUSTER],
                                                      batch_perplex=r[engine.PPL_BATCH],
                                                      shape_perplex=r[engine.PPL_SHAPE]))
        emission_loss = recs[:, engine.EM].sum() / num_strings
        end_prediction_loss = recs[:, engine.OFF].sum() / num_strings
        kl_loss = recs[:, engine.KL].sum() / num_strings
        mean_loss = emission_loss + end_prediction_loss + kl_loss
        logger.info("mean training emission negative pdf loss (per string): {:5.4f}".format(emission_loss))
        logger.info("mean training end-prediction loss (per string): {:5.4f}".format(end_prediction_loss))
        logger.info("mean training KL (per string): {:5.4f}".format(kl_loss))
        logger.info("mean training total loss (per string): {:5.4f}".format(mean_loss))
        if hasattr(self.feature_sampler, "update_epoch_init_iter_counts"):
            self.feature_sampler.update_epoch_init_iter_counts()
        self.last_train = dict(em=emission_loss, off=end_prediction_loss, kl=kl_loss, total=mean_loss,
                               batch_loss=list(recs[:, engine.LOSS]),
                               perplex=recs[:, engine.PPL_CLUSTER:engine.PPL_SHAPE + 1].tolist())
        return mean_loss

    def test_or_validate(self, dataloader, is_pretraining=False):
        """learning.py:200-240 (no weight update; still samples)."""
        self.encoder.eval()
        self.feature_sampler.eval()
        self.decoder.eval()
        num_batches = dataloader.get_num_batches()
        num_strings = len(dataloader.dataset)
        records = []
        with torch.no_grad():
            for batch_ix, (packed_input, is_offset, speaker, _) in enumerate(dataloader, 1):
                b_global = int(packed_input.batch_sizes[0])
                shard = self._shard(packed_input, is_offset, speaker)
                if shard is None:
                    records.append(torch.zeros_like(self.step.scalars))
                    continue
                data, bsz, off, spk = self._to_device(*shard)
                sc, _ = self.step.forward_backward(data, bsz, off, spk, num_strings, is_pretraining=is_pretraining,
                                                   train=False, loss_batch=b_global)
                records.append(sc.clone())
                logger.info("{batch_ix}/{num_batches} validation batches complete.".format(
                    batch_ix=batch_ix, num_batches=num_batches))
        recs = torch.stack(records)
        if self.world > 1:
            dist.all_reduce(recs, op=dist.ReduceOp.SUM)
        recs = recs.cpu()
        engine.check_status(recs, "validation batch")
        recs = recs.double().numpy()
        emission_loss = recs[:, engine.EM].sum() / num_strings
        end_prediction_loss = recs[:, engine.OFF].sum() / num_strings
        kl_loss = recs[:, engine.KL].sum() / num_strings
        mean_loss = emission_loss + end_prediction_loss + kl_loss
        logger.info("mean validation emission negative pdf loss (per string): {:5.4f}".format(emission_loss))
        logger.info("mean validation end-prediction loss (per string): {:5.4f}".format(end_prediction_loss))
        logger.info("mean validation KL (per string): {:5.4f}".format(kl_loss))
        logger.info("mean validation total loss (per string): {:5.4f}".format(mean_loss))
        self.last_valid = dict(em=emission_loss, off=end_prediction_loss, kl=kl_loss, total=mean_loss)
        return mean_loss

    def learn(self, train_dataset, valid_dataset, num_epochs, batch_size_train, batch_size_valid, pretrain_epochs=0,
              learning_rate=0.1, momentum=0.9, gradient_clip=0.25, patience=0, featurizer=None):
        """learning.py:245-290.  featurizer: a data_utils.DeviceFeaturizer when the
        datasets return raw samples (--gpu_featurize)."""
        # single device: RandomSampler draws from the global CPU generator as in
        # the reference (bit-exact batch order).  Data parallel: a generator of
        # its own, seeded alike on every rank, so every rank shuffles -- and
        # shards -- the same global batches whatever else uses the CPU RNG
        # The generator's seed and state travel in the checkpoint, so a resumed
        # run continues the shuffle sequence instead of replaying epoch 1's.
        gen = None
        if self.world > 1:
            gen = torch.Generator().manual_seed(self.seed)
            state = self.checkpoint.get("dp_shuffle_state") if self.retrieval else None
            if state is not None:
                gen.set_state(state)
        self._shuffle_gen = gen
        train_dataloader = data_utils.DataLoader(train_dataset, batch_size=batch_size_train, shuffle=True,
                                                 featurizer=featurizer, generator=gen)
        valid_dataloader = data_utils.DataLoader(valid_dataset, batch_size=batch_size_valid, featurizer=featurizer)
        self.optimizer = torch.optim.SGD(self.parameters(), lr=learning_rate, momentum=momentum)
        if self.retrieval:
            initial_epoch = self.last_epoch + 1
            logger.info("To be restarted from the beginning of epoch #: {epoch}".format(epoch=initial_epoch))
            self.optimizer.load_state_dict(self.checkpoint["optimizer"])
            self.lr_scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(self.optimizer)
            self.lr_scheduler.load_state_dict(self.checkpoint["lr_scheduler"])
            self._restore_momentum()
        else:
            self.lr_scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(self.optimizer, patience=patience)
            logger.info("START LEARNING.")
            logger.info("max # of epochs: {ep}".format(ep=num_epochs))
            logger.info("first {} epochs are for pretraining w/o gumbel-softmax sampling.".format(pretrain_epochs))
            logger.info("batch size for training data: {size}".format(size=batch_size_train))
            logger.info("batch size for validation data: {size}".format(size=batch_size_valid))
            logger.info("initial learning rate: {lr}".format(lr=learning_rate))
            logger.info("momentum for SGD: {momentum}".format(momentum=momentum))
            self.gradient_clip = gradient_clip
            logger.info("gradient clipping: {gc}".format(gc=self.gradient_clip))
            initial_epoch = 1
        self.history = []
        for epoch in range(initial_epoch, num_epochs + 1):
            logger.info("START OF EPOCH: {:3d}".format(epoch))
            logger.info("current learning rate: {lr}".format(lr=self.optimizer.param_groups[0]["lr"]))
            is_pretrain = epoch <= pretrain_epochs
            logger.info("start of TRAINING phase.")
            self.train(train_dataloader, is_pretrain)
            logger.info("end of TRAINING phase.")
            logger.info("start of VALIDATION phase.")
            mean_valid_loss = self.test_or_validate(valid_dataloader, is_pretrain)
            logger.info("end of VALIDATION phase.")
            self.history.append(dict(epoch=epoch, train=self.last_train, valid=self.last_valid))
            self.lr_scheduler.step(mean_valid_loss)
            if epoch == pretrain_epochs:
                self.lr_scheduler.best = math.inf  # delete the best during pretraining (learning.py:284-286)
                logger.info("END OF PRETRAINING.")
            self.save_model(epoch)
            logger.info("END OF EPOCH: {:3d}".format(epoch))
        logger.info("END OF TRAINING")

    def _restore_momentum(self):
        st = self.optimizer.state
        bufs = [st[p].get("momentum_buffer") for p in self.step.flat.params] if st else []
        if bufs and all(b is not None for b in bufs):
            self.step.momentum_buf = torch.cat([b.reshape(-1).to(self.device) for b in bufs])
            self.step.momentum_init = False
            self._momentum_views()

    def save_model(self, epoch):
        """learning.py:293-314 (same keys; plus the Philox noise state).  Under
        data parallelism the stored Philox offset is the maximum over the ranks,
        so a resumed rank never re-draws counters it already used."""
        nstate = noise.get_state()
        if self.world > 1:
            o = torch.tensor([nstate["offset"]], dtype=torch.int64, device=self.device)
            dist.all_reduce(o, op=dist.ReduceOp.MAX)
            nstate["offset"] = int(o)
        if self.rank != 0:
            return
        self._momentum_views()
        checkpoint = {
            "epoch": epoch,
            "encoder": self.encoder.state_dict(),
            "encoder_init_parameters": self.encoder.pack_init_parameters(),
            "feature_sampler": self.feature_sampler.state_dict(),
            "feature_sampler_init_parameters": self.feature_sampler.pack_init_parameters(),
            "decoder": self.decoder.state_dict(),
            "decoder_init_parameters": self.decoder.pack_init_parameters(),
            "optimizer": self.optimizer.state_dict(),
            "lr_scheduler": self.lr_scheduler.state_dict(),
            "gradient_clip": self.gradient_clip,
            "random_state": torch.get_rng_state(),
            "abcd_noise_state": nstate,
            "seed": self.seed,
        }
        if getattr(self, "_shuffle_gen", None) is not None:
            checkpoint["dp_shuffle_state"] = self._shuffle_gen.get_state()
        if torch.cuda.is_available():
            checkpoint["random_state_cuda"] = torch.cuda.get_rng_state_all()
        torch.save(checkpoint, os.path.join(self.save_dir, "checkpoint.pt"))
        logger.info("Config successfully saved.")

    def retrieve_model(self, checkpoint_path=None, device="cuda"):
        """learning.py:317-347 -- also loads checkpoints written by the reference."""
        _check_device(device)
        self.device = torch.device(device)
        if checkpoint_path is None:
            checkpoint_path = os.path.join(self.save_dir, "checkpoint.pt")
        self.checkpoint = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        self.encoder = model.RNN_Variational_Encoder(**self.checkpoint["encoder_init_parameters"])
        self.feature_sampler = model.ABCDSampler(**self.checkpoint["feature_sampler_init_parameters"])
        self.decoder = model.RNN_Variational_Decoder(**self.checkpoint["decoder_init_parameters"])
        self.encoder.load_state_dict(self.checkpoint["encoder"], strict=False)
        self.feature_sampler.load_state_dict(self.checkpoint["feature_sampler"])
        self.decoder.load_state_dict(self.checkpoint["decoder"])
        if not hasattr(self, "rank"):
            self.rank, self.world = parallel.world()
        self._finish_modules()
        self.gradient_clip = self.checkpoint["gradient_clip"]
        # the run's seed (reference checkpoints carry none: the CLI default)
        self.seed = int(self.checkpoint.get("seed", 1111))
        try:
            torch.set_rng_state(self.checkpoint["random_state"])
        except RuntimeError:
            logger.warning("Failed to retrieve random_state.")
        if "abcd_noise_state" in self.checkpoint:
            noise.set_state(self.checkpoint["abcd_noise_state"], rank=self.rank)
        if "random_state_cuda" in self.checkpoint:
            try:
                torch.cuda.set_rng_state_all(self.checkpoint["random_state_cuda"])
            except Exception:
                pass
        return self.checkpoint["epoch"]


def get_parameters(argv=None):
    """learning.py:351-394 (+ --noise)."""
    p = argparse.ArgumentParser()
    p.add_argument("input_root", type=str, help="Path to the root directory under which inputs are located.")
    p.add_argument("annotation_file", type=str, help="Path to the annotation csv file.")
    p.add_argument("--annotation_sep", type=str, default=",", help="Separator symbol of the annotation file.")
    p.add_argument("-S", "--save_root", type=str, default=None, help="Path to the directory where results are saved.")
    p.add_argument("-j", "--job_id", type=str, default="NO_JOB_ID", help="Job ID. For users of computing clusters.")
    p.add_argument("-s", "--seed", type=int, default=1111, help="random seed")
    p.add_argument("-d", "--device", type=str, default="cuda", help="Computing device (GPU only).")
    p.add_argument("-e", "--epochs", type=int, default=20, help="# of epochs to train the model.")
    p.add_argument("--pretrain_epochs", type=int, default=5,
                   help="# of initial epochs to pretrain the model w/o gumbel-softmax sampling.")
    p.add_argument("-b", "--batch_size", type=int, default=512, help="Batch size for training.")
    p.add_argument("--validation_batch_size", type=int, default=None, help="Batch size for validation.")
    p.add_argument("-l", "--learning_rate", type=float, default=1.0, help="Initial learning rate.")
    p.add_argument("-M", "--momentum", type=float, default=0.0, help="Momentum for the stochastic gradient descent.")
    p.add_argument("-c", "--clip", type=float, default=1.0, help="Gradient clipping.")
    p.add_argument("-p", "--patience", type=int, default=0, help="# of epochs before updating the learning rate.")
    p.add_argument("-R", "--encoder_rnn_type", type=str, default="LSTM", help="Name of RNN for the encoder.")
    p.add_argument("--decoder_rnn_type", type=str, default=None, help="Name of RNN for the decoder.")
    p.add_argument("-K", "--num_feature_categories", type=int, default=128, help="# of discrete categories.")
    p.add_argument("-f", "--feature_dim", type=int, default=256, help="# of dimensions of the codebook vectors.")
    p.add_argument("--encoder_rnn_layers", type=int, default=1, help="# of hidden layers in the encoder RNN.")
    p.add_argument("--encoder_rnn_hidden_size", type=int, default=256, help="# of RNN units in the encoder.")
    p.add_argument("--decoder_rnn_hidden_size", type=int, default=256, help="# of RNN units in the decoder.")
    p.add_argument("--mlp_hidden_size", type=int, default=256, help="# of neurons in the MLP hidden layers.")
    p.add_argument("--speaker_embed_dim", type=int, default=None, help="Speaker embedding dim fed to the decoder.")
    p.add_argument("--encoder_hidden_dropout", type=float, default=0.0, help="Dropout in non-top encoder layers.")
    p.add_argument("--decoder_input_dropout", type=float, default=0.0, help="Dropout in the decoder input.")
    p.add_argument("--greedy_decoder", action="store_true", help="Decoder receives no self-feedback.")
    p.add_argument("--esn_leak", type=float, default=1.0, help="Leak for the echo-state network (unsupported).")
    p.add_argument("--unidirectional_encoder", action="store_true", help="The RNN encoder is unidirectional.")
    p.add_argument("--bidirectional_decoder", action="store_true", help="(unsupported: broken in the reference)")
    p.add_argument("--right2left_decoder_weight", type=float, default=0.5, help="(bidirectional decoder only)")
    p.add_argument("--fft_frame_length", type=float, default=0.008, help="FFT frame length in sec.")
    p.add_argument("--fft_step_size", type=float, default=0.004, help="FFT step size in sec.")
    p.add_argument("--fft_window_type", type=str, default="hann_window", help="Window type for FFT.")
    p.add_argument("--fft_no_centering", action="store_true", help="If selected, no centering in FFT.")
    p.add_argument("--channel", type=int, default=0, help="Channel ID # of multichannel recordings to use.")
    p.add_argument("-N", "--data_normalizer", type=float, default=1.0, help="Normalizing constant.")
    p.add_argument("-E", "--epsilon", type=float, default=2 ** (-15), help="Added before log.")
    p.add_argument("--prior_concentration", type=float, default=1.0, help="Dirichlet prior concentration.")
    p.add_argument("--noise", type=str, default="philox", choices=["philox", "reference"],
                   help="philox: in-kernel noise (default); reference: host torch CPU generator in the "
                        "reference's order (bit-identical noise to a reference CPU run).")
    p.add_argument("--gpu_featurize", action="store_true",
                   help="STFT + log + packing of each batch on the GPU (libabcd_hip) instead of per item on the "
                        "host; same batches, features within fp32 FFT noise.")
    return p.parse_args(argv)


def get_save_dir(save_root, job_id_str):
    save_dir = os.path.join(save_root, job_id_str)
    if not os.path.isdir(save_dir):
        os.makedirs(save_dir, exist_ok=True)
    return save_dir


def init_distributed():
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and not dist.is_initialized():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        return f"cuda:{local}"
    return None


def main(argv=None):
    parameters = get_parameters(argv)
    dev = init_distributed()
    if dev is not None:
        parameters.device = dev
    save_root = parameters.save_root if parameters.save_root is not None else parameters.input_root
    save_dir = get_save_dir(save_root, parameters.job_id)
    speaker_coding_path = os.path.join(save_dir, "speaker_coding.json")
    speaker2ix = None
    if os.path.isfile(speaker_coding_path):
        with open(speaker_coding_path, "r") as f:
            speaker2ix = json.load(f)
    data_parser = data_utils.Data_Parser(parameters.input_root, parameters.annotation_file,
                                         annotation_sep=parameters.annotation_sep, speaker2ix=speaker2ix)
    fs = data_parser.get_sample_freq()
    num_speakers = data_parser.get_num_speakers()
    if num_speakers > 0 and speaker2ix is None and parallel.world()[0] == 0:
        with open(speaker_coding_path, "w") as f:
            json.dump(data_parser.speaker2ix, f)
    fft_frame_length = int(np.floor(parameters.fft_frame_length * fs))
    fft_step_size = int(np.floor(parameters.fft_step_size * fs))
    if parameters.decoder_rnn_type is None:
        parameters.decoder_rnn_type = parameters.encoder_rnn_type
    learner = Learner(int(fft_frame_length / 2 + 1), parameters.encoder_rnn_hidden_size,
                      parameters.decoder_rnn_hidden_size, parameters.mlp_hidden_size,
                      parameters.num_feature_categories, parameters.feature_dim, save_dir,
                      encoder_rnn_type=parameters.encoder_rnn_type, decoder_rnn_type=parameters.decoder_rnn_type,
                      encoder_rnn_layers=parameters.encoder_rnn_layers,
                      encoder_hidden_dropout=parameters.encoder_hidden_dropout,
                      decoder_input_dropout=parameters.decoder_input_dropout, device=parameters.device,
                      seed=parameters.seed, decoder_self_feedback=not parameters.greedy_decoder,
                      bidirectional_encoder=not parameters.unidirectional_encoder,
                      bidirectional_decoder=parameters.bidirectional_decoder,
                      right2left_decoder_weight=parameters.right2left_decoder_weight, num_speakers=num_speakers,
                      speaker_embed_dim=parameters.speaker_embed_dim,
                      prior_concentration=parameters.prior_concentration, noise_mode=parameters.noise)
    to_tensor = data_utils.ToTensor()
    stft = data_utils.STFT(fft_frame_length, fft_step_size, window=parameters.fft_window_type,
                           centering=not parameters.fft_no_centering)
    eps, norm = parameters.epsilon, parameters.data_normalizer
    log_and_normalize = data_utils.Transform(lambda x: (x + eps).log() / norm)
    logger.info("log(abs(STFT(wav))) + {eps}) / {normalizer} will be the input.".format(eps=eps, normalizer=norm))
    logger.info("Sampling frequency of data: {fs}".format(fs=fs))
    logger.info("STFT window type: {w}".format(w=parameters.fft_window_type))
    logger.info("STFT frame lengths: {v} sec".format(v=parameters.fft_frame_length))
    logger.info("STFT step size: {v} sec".format(v=parameters.fft_step_size))
    featurizer = None
    transform = Compose([to_tensor, stft, log_and_normalize])
    if parameters.gpu_featurize:
        featurizer = data_utils.DeviceFeaturizer(fft_frame_length, fft_step_size, window=parameters.fft_window_type,
                                                 centering=not parameters.fft_no_centering, eps=eps, normalizer=norm,
                                                 device=parameters.device)
        transform = None
        logger.info("STFT featurisation and packing on the GPU.")
    train_dataset = data_parser.get_data(data_type="train", transform=transform, channel=parameters.channel)
    valid_dataset = data_parser.get_data(data_type="valid", transform=transform, channel=parameters.channel)
    if parameters.validation_batch_size is None:
        parameters.validation_batch_size = parameters.batch_size
    learner.learn(train_dataset, valid_dataset, parameters.epochs, parameters.batch_size,
                  parameters.validation_batch_size, pretrain_epochs=parameters.pretrain_epochs,
                  learning_rate=parameters.learning_rate, momentum=parameters.momentum,
                  gradient_clip=parameters.clip, patience=parameters.patience, featurizer=featurizer)
    return learner


if __name__ == "__main__":
    main()
