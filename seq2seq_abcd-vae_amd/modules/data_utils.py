# coding: utf-8
"""Host-side data pipeline with the reference API (ABCD-VAE/modules/data_utils.py).

CSV annotation + WAV -> STFT amplitude -> log(x + eps) / N -> length-sorted
PackedSequence.  This is the hot path's INPUT CONTRACT:
batches are popped from the END of the BatchSampler list, sorted by length
(desc) inside the batch, and `is_offset` marks each segment's last frame.  The
sampler draws from torch's global CPU generator exactly like the reference,
so epoch/batch order matches a reference run with the same seed.

Differences from the reference are compatibility fixes only (the reference
targets PyTorch 1.2 / pandas 1.x): frame indices are kept as int, and
`Tensor.stft` is called with `return_complex=True` and turned into the same
real-pair amplitude.
"""
import collections
import os.path

import numpy as np
import pandas as pd
import scipy.io.wavfile as spw
import torch
import torch.utils.data


class Data_Parser(object):
    """data_utils.py:10-57"""

    def __init__(self, input_root, annotation_file, data_type_col_name="data_type", annotation_sep=",",
                 speaker2ix=None):
        self.df_annotation = pd.read_csv(annotation_file, sep=annotation_sep)
        self.input_root = input_root
        self.data_type_col_name = data_type_col_name
        self.index_speakers(speaker2ix)

    def index_speakers(self, speaker2ix):
        if "speaker" in self.df_annotation.columns:
            self.df_annotation["speaker"] = self.df_annotation["speaker"].astype(str)
            if speaker2ix is None:
                self.speaker2ix = {spk: ix for ix, spk in enumerate(self.df_annotation.speaker.unique())}
            else:
                self.speaker2ix = speaker2ix
        else:
            self.speaker2ix = None

    def get_num_speakers(self):
        return 0 if self.speaker2ix is None else len(self.speaker2ix)

    def get_data(self, data_type=None, transform=None, channel=0):
        if data_type is None:
            sub_df = self.df_annotation.copy()
        else:
            sub_df = self.df_annotation[self.df_annotation[self.data_type_col_name] == data_type].copy()
        return Dataset(sub_df, self.input_root, transform=transform, channel=channel, speaker2ix=self.speaker2ix)

    def get_sample_freq(self, input_path=None):
        if input_path is None:
            input_path = self.df_annotation.loc[0, "input_path"]
        fs, _ = spw.read(os.path.join(self.input_root, input_path))
        return fs


class Dataset(torch.utils.data.Dataset):
    """data_utils.py:60-103"""

    def __init__(self, df_annotation, input_root, transform=None, channel=0, speaker2ix=None):
        self.df_annotation = df_annotation
        self.input_root = input_root
        self.transform = transform
        self.channel = channel
        self.speaker2ix = speaker2ix
        self._wav_cache = collections.OrderedDict()
        self.get_discrete_bounds()

    def get_discrete_bounds(self):
        onset = np.zeros(len(self.df_annotation), dtype=np.int64)
        offset = np.zeros(len(self.df_annotation), dtype=np.int64)
        pos = {ix: i for i, ix in enumerate(self.df_annotation.index)}
        for input_path, sub_df in self.df_annotation.groupby("input_path"):
            fs, _ = spw.read(os.path.join(self.input_root, input_path))
            for ix, on, off in zip(sub_df.index, (sub_df.onset * fs).round(), (sub_df.offset * fs).round()):
                onset[pos[ix]] = int(on)
                offset[pos[ix]] = int(off)
        self.df_annotation["onset_ix"] = onset
        self.df_annotation["offset_ix"] = offset
        self.df_annotation["length"] = offset - onset

    def sort_indices_by_length(self, ixs):
        return self.df_annotation.iloc[ixs, :].sort_values("length", ascending=False).index

    def __len__(self):
        return self.df_annotation.shape[0]

    WAV_CACHE_FILES = 64  # open recordings kept (memory-mapped: the page cache holds the bytes)

    def _read(self, input_path):
        # the reference re-reads the WAV for every item (data_utils.py:91); a small LRU of
        # memory-mapped recordings gives identical samples without the repeated I/O and
        # without holding whole corpora in process memory
        cache = self._wav_cache
        if input_path in cache:
            cache.move_to_end(input_path)
            return cache[input_path]
        path = os.path.join(self.input_root, input_path)
        try:
            data = spw.read(path, mmap=True)[1]
        except ValueError:  # formats scipy cannot map (e.g. 24-bit PCM): read into memory
            data = spw.read(path)[1]
        cache[input_path] = data
        if len(cache) > self.WAV_CACHE_FILES:
            cache.popitem(last=False)
        return data

    def __getitem__(self, ix):
        row = self.df_annotation.loc[ix]
        input_data = self._read(row["input_path"])
        if input_data.ndim > 1:
            input_data = input_data[:, self.channel]
        input_data = input_data[int(row["onset_ix"]):int(row["offset_ix"])].astype(np.float32)
        if self.speaker2ix is None:
            speaker = float("nan")
        else:
            speaker = self.speaker2ix[row["speaker"]]
        if self.transform:
            input_data = self.transform(input_data)
        return input_data, speaker


class ToTensor(object):
    def __call__(self, input_data):
        return torch.from_numpy(input_data)


class Transform(object):
    def __init__(self, in_trans):
        self.in_trans = in_trans

    def __call__(self, input_data):
        return self.in_trans(input_data)


class STFT(object):
    """data_utils.py:124-139: |STFT| with time as dim 0."""

    def __init__(self, frame_length, step_size, window="hann_window", centering=True):
        self.frame_length = frame_length
        self.step_size = step_size
        self.window = getattr(torch, window)(frame_length)
        self.centering = centering

    def __call__(self, input_data):
        z = input_data.stft(self.frame_length, hop_length=self.step_size, window=self.window,
                            center=self.centering, return_complex=True)
        return torch.view_as_real(z).pow(2).sum(-1).sqrt().transpose(0, 1).contiguous()


class Compose(object):
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, data):
        for trans in self.transforms:
            data = trans(data)
        return data


class DeviceFeaturizer(object):
    """STFT -> |.| -> log(x + eps) / norm -> pack_sequence for a whole batch on the
    GPU (libabcd_hip: abcd_featurize_packed), replacing the per-item host chain
    ``Compose([ToTensor(), STFT(...), log_and_normalize])`` + ``pack_sequence``
    (data_utils.py:124-139, 165-182; learning.py:456-466).  Takes the RAW
    per-item float32 samples (a Dataset built with transform=None) in packed
    (length-descending) order; returns (packed data L x F on `device`,
    batch_sizes (CPU int64), packed is_offset on `device`)."""

    def __init__(self, frame_length, step_size, window="hann_window", centering=True, eps=2 ** (-15),
                 normalizer=1.0, device="cuda"):
        self.n_fft, self.hop, self.center = int(frame_length), int(step_size), bool(centering)
        self.eps, self.norm = float(eps), float(normalizer)
        self.device = torch.device(device)
        self.window = getattr(torch, window)(self.n_fft).to(self.device, torch.float32).contiguous()
        self._ws = None

    def num_frames(self, length):
        from . import _native as N
        return int(N.lib().abcd_stft_frames(int(length), self.n_fft, self.hop, int(self.center)))

    def __call__(self, waves):
        from . import _native as N
        lib = N.lib()
        lens = [int(len(w)) for w in waves]
        frames = [self.num_frames(n) for n in lens]
        if any(f <= 0 for f in frames) or any(a < b for a, b in zip(frames, frames[1:])):
            raise ValueError("segments must be in length-descending order and long enough for one frame")
        T, B = frames[0], len(waves)
        batch_sizes = torch.tensor([sum(f > t for f in frames) for t in range(T)], dtype=torch.int64)
        L = int(batch_sizes.sum())
        F = self.n_fft // 2 + 1
        host = torch.from_numpy(np.concatenate([np.asarray(w, dtype=np.float32) for w in waves]))
        wave = host.pin_memory().to(self.device, non_blocking=True) if self.device.type == "cuda" else host
        seg_off = np.cumsum([0] + lens[:-1]).astype(np.int64)
        seg_len = np.asarray(lens, dtype=np.int64)
        out = torch.empty(L, F, device=self.device)
        is_off = torch.empty(L, device=self.device)
        nbytes = lib.abcd_featurize_workspace_bytes(B, T)
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = N.workspace(2 * nbytes, self.device)
        N.check(lib.abcd_featurize_packed(N.ptr(wave), seg_off.ctypes.data, seg_len.ctypes.data, B, self.n_fft,
                                          self.hop, int(self.center), N.ptr(self.window), self.eps, self.norm,
                                          batch_sizes.data_ptr(), T, L, N.ptr(out), N.ptr(is_off), N.ptr(self._ws),
                                          self._ws.numel(), N.stream()), "featurize")
        return out, batch_sizes, is_off


class DataLoader(object):
    """data_utils.py:150-185: yields (PackedSequence, packed is_offset, speakers, ixs).

    With ``featurizer`` (a DeviceFeaturizer) the dataset must return raw
    samples (transform=None) and the whole batch is featurised and packed on
    the GPU; batch order, in-batch sort and outputs are those of the host path."""

    def __init__(self, dataset, batch_size=1, shuffle=False, featurizer=None, generator=None):
        self.dataset = dataset
        self.featurizer = featurizer
        self.shuffle = shuffle
        if shuffle:
            sampler = torch.utils.data.RandomSampler(self.dataset, replacement=False, generator=generator)
        else:
            sampler = torch.utils.data.SequentialSampler(self.dataset)
        self.batch_sampler = torch.utils.data.BatchSampler(sampler, batch_size, drop_last=False)

    def __iter__(self):
        self.batches = list(self.batch_sampler)
        return self

    def __next__(self):
        if not self.batches:
            raise StopIteration
        ixs = self.batches.pop()
        ixs = self.dataset.sort_indices_by_length(ixs)
        if self.featurizer is not None:
            waves, speakers = [], []
            for ix in ixs:
                w, spk = self.dataset[ix]
                waves.append(w)
                speakers.append(spk)
            data, batch_sizes, is_off = self.featurizer(waves)
            packed = torch.nn.utils.rnn.PackedSequence(data, batch_sizes)
            return packed, torch.nn.utils.rnn.PackedSequence(is_off, batch_sizes), torch.tensor(speakers), ixs
        batched_input, speakers, is_offset = [], [], []
        for ix in ixs:
            seq, spk = self.dataset[ix]
            batched_input.append(seq)
            speakers.append(spk)
            is_offset.append(torch.tensor([0.0] * (seq.size(0) - 1) + [1.0]))
        batched_input = torch.nn.utils.rnn.pack_sequence(batched_input)
        is_offset = torch.nn.utils.rnn.pack_sequence(is_offset)
        speakers = torch.tensor(speakers)
        return batched_input, is_offset, speakers, ixs

    def get_num_batches(self):
        return len(self.batch_sampler)
