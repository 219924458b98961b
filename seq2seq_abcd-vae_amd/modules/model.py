# coding: utf-8
"""nn.Module surface of the reference model (ABCD-VAE/modules/model.py), backed
by the MI355X kernels of libabcd_hip.so.

Class names, constructor signatures, ``forward``/``sample``/``kl_divergence``
signatures, attribute names, ``state_dict`` keys and ``pack_init_parameters``
dicts follow the reference (file:line cited per class) so that ``learning.py``,
``encode*.py`` and reference checkpoints work unchanged.  Parameters are
created with the same torch init calls in the same order as the reference, so
``torch.manual_seed(seed)`` gives bit-identical initial weights.

Every forward/backward runs on the GPU through the ``abcd::`` custom operators
of ``ops.py`` (the C ABI registered with ``torch.library``, autograd formulas
included); there is no CPU fallback -- a CPU tensor raises.
"""
import math

import torch

from . import _native as N
from . import noise as _noise
from . import ops
from . import padding as _pad


def _module_pad(module, kind):
    """The module's padded twin (padding.ModulePad) when one of its sizes is
    not a multiple of 16, else None; built once per module."""
    mp = module.__dict__.get("_abcd_mpad", False)
    if mp is False:
        dims = {"encoder": _pad.encoder_dims, "sampler": _pad.sampler_dims, "decoder": _pad.decoder_dims}[kind]
        mp = _pad.ModulePad(kind, module) if dims(module).active else None
        module.__dict__["_abcd_mpad"] = mp
    return mp


# ----------------------------------------------------------------------------
# reference helper functions (model.py:6-37), torch-level, used only on
# tensors the caller already holds (e.g. Sampler.log_pdf in user code)
# ----------------------------------------------------------------------------
def choose_distribution(distribution_name):
    distributions = {"isotropic_gaussian": (sample_from_isotropic_gaussian, log_pdf_isotropic_gaussian,
                                            kl_isotropic_to_standard_gaussian, 2)}
    return distributions[distribution_name]


def sample_from_isotropic_gaussian(mean, log_variance):
    return mean + (0.5 * log_variance).exp() * torch.randn_like(mean)


def kl_isotropic_to_standard_gaussian(mean, log_variance):
    return -0.5 * (1 + log_variance - mean.pow(2) - log_variance.exp()).sum()


def log_pdf_isotropic_gaussian(value, mean, log_variance):
    d = value - mean
    return -0.5 * (math.log(2 * math.pi) + log_variance + d * (-log_variance).exp() * d).sum()


def _packed_struct(data, batch_sizes, F):
    bs = batch_sizes
    if bs.dtype != torch.int64 or bs.device.type != "cpu":
        bs = bs.to("cpu", torch.int64)
    bs = bs.contiguous()
    st = N.Packed()
    st.data = data.data_ptr() if data is not None else None
    st.batch_sizes = bs.data_ptr()
    st.T = int(bs.numel())
    st.L = int(data.shape[0]) if data is not None else int(bs.sum())
    st.B = int(bs[0])
    st.F = int(F)
    return st, bs  # keep bs alive while the struct is used


def _f32c(t):
    if t.dtype != torch.float32:
        raise TypeError(f"fp32 tensors only (got {t.dtype})")
    return t.contiguous()


# ----------------------------------------------------------------------------
# parameter containers with the reference's names / init
# ----------------------------------------------------------------------------
class PackedRNN(torch.nn.Module):
    """Parameter holder standing in for ``torch.nn.LSTM/GRU`` inside the
    encoder (``model.py:53``): same attribute names (mode, input_size,
    hidden_size, num_layers, dropout, bidirectional, batch_first), same
    parameter names/order and the same ``reset_parameters`` (every weight
    U(-1/sqrt(H), 1/sqrt(H)) in ``_flat_weights`` order)."""

    def __init__(self, mode, input_size, hidden_size, num_layers=1, dropout=0.0, bidirectional=False,
                 batch_first=True):
        super().__init__()
        if mode not in ("LSTM", "GRU"):
            raise NotImplementedError(f"rnn_type {mode!r}: only LSTM and GRU run on the HIP path "
                                      "(ESN is broken in the reference on torch>=1.9: torch.eig)")
        self.mode = mode
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.num_layers = num_layers
        self.dropout = float(dropout)
        self.bidirectional = bidirectional
        self.batch_first = batch_first
        G = 4 if mode == "LSTM" else 3
        dirs = 2 if bidirectional else 1
        for l in range(num_layers):
            In = input_size if l == 0 else hidden_size * dirs
            for d in range(dirs):
                sfx = "_reverse" if d == 1 else ""
                self.register_parameter(f"weight_ih_l{l}{sfx}", torch.nn.Parameter(torch.empty(G * hidden_size, In)))
                self.register_parameter(f"weight_hh_l{l}{sfx}",
                                        torch.nn.Parameter(torch.empty(G * hidden_size, hidden_size)))
                self.register_parameter(f"bias_ih_l{l}{sfx}", torch.nn.Parameter(torch.empty(G * hidden_size)))
                self.register_parameter(f"bias_hh_l{l}{sfx}", torch.nn.Parameter(torch.empty(G * hidden_size)))
        self.reset_parameters()

    def reset_parameters(self):
        stdv = 1.0 / math.sqrt(self.hidden_size)
        for w in self.parameters():
            torch.nn.init.uniform_(w, -stdv, stdv)

    def layer_weights(self, l, d):
        sfx = "_reverse" if d == 1 else ""
        return [getattr(self, f"{n}_l{l}{sfx}") for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]


class MLP(torch.nn.Module):
    """``model.py:316-334``: Linear -> Tanh -> Linear (``whole_network``)."""

    def __init__(self, input_size, hidden_size, output_size):
        super().__init__()
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.output_size = output_size
        self.whole_network = torch.nn.Sequential(torch.nn.Linear(input_size, hidden_size), torch.nn.Tanh(),
                                                 torch.nn.Linear(hidden_size, output_size))

    def weights(self):
        return (self.whole_network[0].weight, self.whole_network[0].bias, self.whole_network[2].weight,
                self.whole_network[2].bias)

    def forward(self, batched_input):
        """Linear -> Tanh -> Linear on the HIP GEMMs (``abcd::linear``), with
        autograd (``abcd::linear_bwd``): the standalone MLP trains like the
        reference's (model.py:332-334).  Inside the training step the MLPs run
        fused into the sampler / decoder kernels instead."""
        x = _f32c(batched_input)
        N.require_gpu(x)
        shp = x.shape
        w1, b1, w2, b2 = self.weights()
        hid = ops.linear(x.reshape(-1, shp[-1]), w1, b1, 1)
        out = ops.linear(hid, w2, b2, 0)
        return out.reshape(*shp[:-1], self.output_size)


class MLP_To_k_Vecs(torch.nn.Module):
    """``model.py:303-314``"""

    def __init__(self, input_size, hidden_size, output_size, k):
        super().__init__()
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.output_size = output_size
        self.k = k
        self.mlps = torch.nn.ModuleList([MLP(input_size, hidden_size, output_size) for _ in range(k)])

    def forward(self, batched_input):
        return [mlp(batched_input) for mlp in self.mlps]


class RNN_Cell(torch.nn.Module):
    """``model.py:287-300``: input dropout + LSTMCell/GRUCell (parameter holder)."""

    def __init__(self, input_size, hidden_size, model_type="LSTM", input_dropout=0.0, esn_leak=1.0):
        super().__init__()
        if model_type not in ("LSTM", "GRU"):
            raise NotImplementedError(f"decoder rnn_type {model_type!r}: only LSTM and GRU are supported")
        self.drop = torch.nn.Dropout(input_dropout)
        self.mode = model_type
        self.cell = getattr(torch.nn, model_type + "Cell")(input_size, hidden_size)

    def forward(self, batched_input, init_hidden=None):
        """One standalone cell step, model.py:297-300: ``cell(drop(x), init_hidden)``.

        The decoder steps its cell inside the fused persistent kernels; this
        is the reference module's own API for other callers.  The two
        projections x W_ih^T + b_ih and h W_hh^T + b_hh run on the HIP GEMMs
        (``abcd::linear``, differentiable); the gate nonlinearities of
        nn.LSTMCell / nn.GRUCell (PyTorch's gate order i, f, g, o / r, z, n)
        are elementwise torch ops on the device."""
        x = _f32c(self.drop(batched_input))
        N.require_gpu(x)
        cell = self.cell
        B, H = x.shape[0], cell.hidden_size
        if init_hidden is None:
            z = x.new_zeros(B, H)
            init_hidden = (z, z) if self.mode == "LSTM" else z
        h = init_hidden[0] if self.mode == "LSTM" else init_hidden
        gi = ops.linear(x, cell.weight_ih, cell.bias_ih, 0)
        gh = ops.linear(_f32c(h), cell.weight_hh, cell.bias_hh, 0)
        if self.mode == "LSTM":
            i, f, g, o = (gi + gh).chunk(4, 1)
            c = torch.sigmoid(f) * init_hidden[1] + torch.sigmoid(i) * torch.tanh(g)
            return torch.sigmoid(o) * torch.tanh(c), c
        ir, iz, inn = gi.chunk(3, 1)
        hr, hz, hn = gh.chunk(3, 1)
        r, zg = torch.sigmoid(ir + hr), torch.sigmoid(iz + hz)
        n = torch.tanh(inn + r * hn)
        return (1 - zg) * n + zg * h


# ----------------------------------------------------------------------------
# Encoder (model.py:40-79)
# ----------------------------------------------------------------------------
class RNN_Variational_Encoder(torch.nn.Module):
    """Bi-directional LSTM/GRU over a PackedSequence; returns the last (h, c)
    of every layer/direction flattened to (B, hidden_size_total)."""

    def __init__(self, input_size, rnn_hidden_size, rnn_type="LSTM", rnn_layers=1, hidden_dropout=0.0,
                 bidirectional=True, esn_leak=1.0):
        super().__init__()
        self.rnn = PackedRNN(rnn_type, input_size, rnn_hidden_size, rnn_layers, dropout=hidden_dropout,
                             bidirectional=bidirectional, batch_first=True)
        self.hidden_size_total = rnn_layers * rnn_hidden_size
        if bidirectional:
            self.hidden_size_total *= 2
        if rnn_type == "LSTM":
            self.hidden_size_total *= 2

    def _cfg(self):
        c = N.EncoderCfg()
        c.input_size, c.hidden_size = self.rnn.input_size, self.rnn.hidden_size
        c.rnn_type = N.LSTM if self.rnn.mode == "LSTM" else N.GRU
        c.layers, c.bidirectional = self.rnn.num_layers, int(self.rnn.bidirectional)
        return c

    def _params(self, grads=None):
        st = N.EncoderParams()
        dirs = 2 if self.rnn.bidirectional else 1
        for l in range(self.rnn.num_layers):
            for d in range(dirs):
                ws = self.rnn.layer_weights(l, d) if grads is None else grads[(l, d)]
                st.w[l][d].w_ih, st.w[l][d].w_hh, st.w[l][d].b_ih, st.w[l][d].b_hh = [
                    None if t is None else t.data_ptr() for t in ws]
        return st

    def draw_dropout_noise(self, L, device):
        """Training-mode inter-layer dropout noise (model.py:53: nn.LSTM/GRU with
        dropout = hidden_dropout), one L x dirs*H tensor per layer boundary in
        layer order -- the reference's RNG order within the step -- or None."""
        p = self.rnn.dropout
        if not (self.training and p > 0 and self.rnn.num_layers > 1):
            return None
        dirs = 2 if self.rnn.bidirectional else 1
        return [_noise.dropout_noise((L, dirs * self.rnn.hidden_size), p, device)
                for _ in range(self.rnn.num_layers - 1)]

    def _cfg_list(self):
        return [self.rnn.input_size, self.rnn.hidden_size, N.LSTM if self.rnn.mode == "LSTM" else N.GRU,
                self.rnn.num_layers, int(self.rnn.bidirectional)]

    def _weights(self):
        dirs = 2 if self.rnn.bidirectional else 1
        return [t for l in range(self.rnn.num_layers) for d in range(dirs) for t in self.rnn.layer_weights(l, d)]

    def forward(self, packed_input):
        data = _f32c(packed_input.data)
        N.require_gpu(data)
        noise = self.draw_dropout_noise(int(data.shape[0]), data.device)
        mp = _module_pad(self, "encoder")
        if mp is None:
            out, _ws = ops.encoder(data, packed_input.batch_sizes, self._weights(), noise or [], self._cfg_list())
            return out
        # hidden size not a multiple of 16: the zero-padded twin (padding.py), real columns out
        d = mp.dims
        noise = [_pad.pad_col_blocks(n, d.dirs, d.H, d.Hp) for n in (noise or [])]
        out, _ws = ops.encoder(data, packed_input.batch_sizes, mp.weights(self._weights()), noise, mp.cfg)
        return out.index_select(1, d.out_cols.to(out.device))

    def pack_init_parameters(self):
        return {"input_size": self.rnn.input_size, "rnn_hidden_size": self.rnn.hidden_size,
                "rnn_type": self.rnn.mode.split("_")[0], "rnn_layers": self.rnn.num_layers,
                "hidden_dropout": self.rnn.dropout, "bidirectional": self.rnn.bidirectional}


# ----------------------------------------------------------------------------
# Samplers (model.py:538-705, plain/modules/model.py:538-567)
# ----------------------------------------------------------------------------
class _SamplerBase(torch.nn.Module):
    """Shared native plumbing of ABCDSampler and the plain feature Sampler."""

    def _mlps(self):
        raise NotImplementedError

    def _scfg(self):
        raise NotImplementedError

    def _sparams(self):
        st = N.SamplerParams()
        for k, m in enumerate(self._mlps()):
            w1, b1, w2, b2 = m.weights()
            st.mlp[k].w1, st.mlp[k].b1, st.mlp[k].w2, st.mlp[k].b2 = (w1.data_ptr(), b1.data_ptr(),
                                                                      w2.data_ptr(), b2.data_ptr())
        if isinstance(self, ABCDSampler):
            st.codebook = self.codebook.data_ptr()
            st.posterior_shape_logits = self.posterior_shape_logits.data_ptr()
            st.prior_concentration = self._prior_value()
        return st

    def _sgrads(self, views):
        """views: dict name -> tensor (mlp{k}.w1 ..., codebook, posterior_shape_logits)."""
        st = N.SamplerGrads()
        for k in range(len(self._mlps())):
            for f in ("w1", "b1", "w2", "b2"):
                t = views.get(f"mlp{k}.{f}")
                setattr(st.mlp[k], f, None if t is None else t.data_ptr())
        for f in ("codebook", "posterior_shape_logits"):
            t = views.get(f)
            setattr(st, f, None if t is None else t.data_ptr())
        return st

    def _ws_for(self, B, device, ws=None):
        nbytes = N.lib().abcd_sampler_workspace_bytes(self._scfg(), B)
        if nbytes == 0:
            raise N.HipError("sampler: unsupported configuration (sizes must be multiples of 16)")
        if ws is None or ws.numel() < nbytes:
            ws = N.workspace(nbytes, device)
        return ws

    def _cfg_list(self):
        c = self._scfg()
        return [c.input_size, c.mlp_hidden, c.num_categories, c.feature_dim, c.plain, c.valid_categories,
                c.valid_feature_dim]

    def _valid(self, c):
        """A padded twin (padding.sampler_twin) carries its model's real (K, D)."""
        vs = self.__dict__.get("valid_sizes")
        if vs is not None:
            # plain: no categories; the real feature dim masks the padding columns' noise (plain_sample)
            c.valid_categories, c.valid_feature_dim = (int(vs[0]), int(vs[1])) if not c.plain else (0, int(vs[1]))
        return c

    def _mlp_weights(self):
        return [t for m in self._mlps() for t in m.weights()]


class ABCDSampler(_SamplerBase):
    """"A"ttention-"B"ased "C"ategorical sampler with a "D"irichlet prior (model.py:538-673)."""

    def __init__(self, input_size, mlp_hidden_size, num_categories, feature_dim, prior_concentration=1.0,
                 min_temperature=1.0, epoch_init_iter_counts=0, temperature_update_freq=1000,
                 temperature_anneal_rate=1e-5):
        super().__init__()
        self.num_categories = num_categories
        self.to_code_like = MLP(input_size, mlp_hidden_size, feature_dim)
        self.min_temperature = min_temperature
        self.epoch_init_iter_counts = epoch_init_iter_counts
        self.iter_counts = epoch_init_iter_counts
        self.temperature_update_freq = temperature_update_freq
        self.temperature_anneal_rate = temperature_anneal_rate
        self.update_temperature((self.iter_counts // self.temperature_update_freq) * self.temperature_update_freq)
        self.register_buffer("prior_concentration", torch.tensor(prior_concentration))
        self.register_parameter("posterior_shape_logits",
                                torch.nn.Parameter(torch.randn(num_categories), requires_grad=True))
        self.register_parameter("codebook", torch.nn.Parameter(torch.randn((feature_dim, num_categories)),
                                                               requires_grad=True))
        self._prior_cache = (None, float(prior_concentration))

    # -- native plumbing --
    def _prior_value(self):
        key = (self.prior_concentration.data_ptr(), self.prior_concentration._version)
        if self._prior_cache[0] != key:
            self._prior_cache = (key, float(self.prior_concentration.detach().cpu()))
        return self._prior_cache[1]

    def _mlps(self):
        return [self.to_code_like]

    def _scfg(self):
        c = N.SamplerCfg()
        c.input_size, c.mlp_hidden = self.to_code_like.input_size, self.to_code_like.hidden_size
        c.num_categories, c.feature_dim, c.plain = self.num_categories, self.to_code_like.output_size, 0
        return self._valid(c)

    def _logit_width(self):
        return self.num_categories

    def _feat_dim(self):
        return self.to_code_like.output_size

    # -- reference API --
    def forward(self, x):
        mp = _module_pad(self, "sampler")
        if mp is None:
            return ops.sampler(_f32c(x), self._mlp_weights(), self.codebook, self._cfg_list())[0]
        d = mp.dims  # a size not a multiple of 16: the zero-padded twin (padding.py)
        lp = ops.sampler(_pad.pad_cols(_f32c(x), d.Ep), mp.weights(self._mlp_weights()), mp.weight(self.codebook),
                         mp.cfg)[0]
        return lp[:, :d.K]

    def sample(self, logits, no_sample=False):
        logits = _f32c(logits)
        N.require_gpu(logits)
        B, K = logits.shape
        mp = _module_pad(self, "sampler")
        width = K if mp is None else mp.dims.Kp
        if no_sample:
            mode, tau, nt, seed, off = N.SAMPLE_SOFTMAX, 1.0, None, 0, 0
        else:
            mode, tau = N.SAMPLE_GUMBEL, float(self.temperature)
            nt, seed, off = _noise.gumbel(B, K, logits.device, width=width)
        if mp is None:
            return ops.sampler_sample(logits, self.codebook, self._cfg_list(), mode, tau, nt, ops._i64(seed),
                                      ops._i64(off))[0]
        feats = ops.sampler_sample(_pad.pad_cols(logits, width), mp.weight(self.codebook), mp.cfg, mode, tau, nt,
                                   ops._i64(seed), ops._i64(off))[0]
        return feats[:, :mp.dims.D]

    def kl_divergence(self, logits, entire_data_size):
        logits = _f32c(logits)
        N.require_gpu(logits)
        mp = _module_pad(self, "sampler")
        if mp is None:
            return ops.sampler_kl(logits, self.posterior_shape_logits, self._cfg_list(), self._prior_value(),
                                  float(entire_data_size))[0]
        return ops.sampler_kl(_pad.pad_cols(logits, mp.dims.Kp), mp.weight(self.posterior_shape_logits), mp.cfg,
                              self._prior_value(), float(entire_data_size))[0]

    def log_pmf(self, targets, logits):
        return torch.nn.functional.cross_entropy(logits, targets, reduction="sum")

    def increment_iter_counts(self):
        self.iter_counts += 1
        if self.iter_counts % self.temperature_update_freq == 0:
            self.update_temperature()

    def update_epoch_init_iter_counts(self):
        self.epoch_init_iter_counts = self.iter_counts

    def update_temperature(self, steps=None):
        if steps is None:
            steps = self.iter_counts
        self.temperature = min(self.min_temperature, math.exp(-self.temperature_anneal_rate * steps))

    def pack_init_parameters(self):
        return {"input_size": self.to_code_like.input_size, "mlp_hidden_size": self.to_code_like.hidden_size,
                "num_categories": self.num_categories, "feature_dim": self.to_code_like.output_size,
                "prior_concentration": self._prior_value(), "min_temperature": self.min_temperature,
                "epoch_init_iter_counts": self.epoch_init_iter_counts,
                "temperature_update_freq": self.temperature_update_freq,
                "temperature_anneal_rate": self.temperature_anneal_rate}


class Sampler(_SamplerBase):
    """``model.py:676-705``.  As the decoder's emission sampler it is a
    parameter holder (the emission MLPs run inside the fused decoder kernels);
    as the plain VAE's feature sampler (``plain/learning.py:90``) forward /
    sample / kl_divergence run on the HIP path."""

    def __init__(self, input_size, mlp_hidden_size, output_size, distribution_name="isotropic_gaussian"):
        super().__init__()
        self.distribution_name = distribution_name
        self._sampler, self._log_pdf, self._kl_divergence, num_parameters = choose_distribution(distribution_name)
        self.to_parameters = MLP_To_k_Vecs(input_size, mlp_hidden_size, output_size, num_parameters)

    def _mlps(self):
        return list(self.to_parameters.mlps)

    def _scfg(self):
        c = N.SamplerCfg()
        c.input_size, c.mlp_hidden = self.to_parameters.input_size, self.to_parameters.hidden_size
        c.num_categories, c.feature_dim, c.plain = 16, self.to_parameters.output_size, 1
        return self._valid(c)

    def _logit_width(self):
        return 2 * self.to_parameters.output_size

    def _feat_dim(self):
        return self.to_parameters.output_size

    def forward(self, parameter_seed):
        f = self.to_parameters.output_size
        mp = _module_pad(self, "sampler")
        if mp is None:
            mv = ops.sampler(_f32c(parameter_seed), self._mlp_weights(), None, self._cfg_list())[0]
            mu, lv = mv[:, :f], mv[:, f:]
        else:  # the zero-padded twin: mv = [mu | 0 | log_var | 0], padding mu = log_var = 0
            fp = mp.dims.Dp
            mv = ops.sampler(_pad.pad_cols(_f32c(parameter_seed), mp.dims.Ep), mp.weights(self._mlp_weights()), None,
                             mp.cfg)[0]
            mu, lv = mv[:, :f], mv[:, fp:fp + f]
        mu._abcd_mv = mv
        return [mu, lv]

    def sample(self, parameters):
        mu, lv = parameters
        mv = getattr(mu, "_abcd_mv", None)
        if mv is None:  # parameters not produced by this module's forward: reference torch formula
            return self._sampler(*parameters)
        B, f = mu.shape
        mp = _module_pad(self, "sampler")
        cfg = self._cfg_list() if mp is None else mp.cfg
        # padding columns (a zero-padded twin's, valid_feature_dim) draw zero noise in both noise modes,
        # so their samples are exactly mu = 0 (plain_sample); only the real f columns are returned
        nt, seed, off = _noise.normal(B, f, mu.device, width=mv.shape[1] // 2)
        return ops.sampler_sample(mv, None, cfg, 0, 1.0, nt, ops._i64(seed), ops._i64(off))[0][:, :f]

    def kl_divergence(self, parameters):
        mu, lv = parameters
        mv = getattr(mu, "_abcd_mv", None)
        if mv is None:
            return self._kl_divergence(*parameters)
        mp = _module_pad(self, "sampler")
        return ops.sampler_kl(mv, None, self._cfg_list() if mp is None else mp.cfg, 1.0, 1.0)[0]

    def log_pdf(self, samples, parameters):
        return self._log_pdf(samples, *parameters)

    def pack_init_parameters(self):
        return {"input_size": self.to_parameters.input_size, "mlp_hidden_size": self.to_parameters.hidden_size,
                "output_size": self.to_parameters.output_size, "distribution_name": self.distribution_name}


# ----------------------------------------------------------------------------
# Decoder (model.py:84-285)
# ----------------------------------------------------------------------------
class RNN_Variational_Decoder(torch.nn.Module):
    """Self-feedback LSTM/GRU decoder with isotropic-Gaussian emission and an
    end-of-segment (offset) predictor, unidirectional (model.py:84-196)."""

    def __init__(self, output_size, rnn_hidden_size, mlp_hidden_size, feature_size,
                 emission_distr_name="isotropic_gaussian", rnn_type="LSTM", rnn_layers=1, input_dropout=0.0,
                 self_feedback=True, bidirectional=False, right2left_weight=0.5, esn_leak=1.0, num_speakers=None,
                 speaker_embed_dim=None):
        super().__init__()
        assert rnn_layers == 1, "Only rnn_layers=1 is currently supported."
        if bidirectional:
            raise NotImplementedError("bidirectional decoder: broken in the reference (model.py:224,258); "
                                      "not on the HIP path")
        if emission_distr_name != "isotropic_gaussian":
            raise NotImplementedError(emission_distr_name)
        if not self_feedback:
            input_dropout = 1.0
        self.bidirectional = False
        self.rnn_type = rnn_type
        self.feature_size = feature_size
        if num_speakers is None or speaker_embed_dim is None:
            self.embed_speaker = None
        else:
            self.embed_speaker = torch.nn.Embedding(num_speakers, speaker_embed_dim, sparse=True)
            feature_size += speaker_embed_dim
        hidden_size_total = rnn_hidden_size * (2 if rnn_type == "LSTM" else 1)
        self.feature2hidden = torch.nn.Linear(feature_size, hidden_size_total)
        self.offset_predictor = MLP(rnn_hidden_size, mlp_hidden_size, 1)
        self.bce_with_logits_loss = torch.nn.BCEWithLogitsLoss(reduction="sum")
        self.emission_sampler = Sampler(rnn_hidden_size, mlp_hidden_size, output_size,
                                        distribution_name=emission_distr_name)
        self.rnn_cell = RNN_Cell(output_size, rnn_hidden_size, model_type=rnn_type, input_dropout=input_dropout,
                                 esn_leak=esn_leak)

    # -- native plumbing --
    def _feedback(self):
        """1: the sample is fed back (eval mode, p < 1); 0: greedy / p = 1 in training (zero input)."""
        return 0 if (self.training and self.rnn_cell.drop.p >= 1.0) else 1

    def _input_dropout_p(self):
        """p of the training-mode input dropout that needs noise (0 < p < 1), else 0."""
        p = self.rnn_cell.drop.p
        return p if (self.training and 0.0 < p < 1.0) else 0.0

    def _dcfg(self, feedback=None):
        c = N.DecoderCfg()
        cell = self.rnn_cell.cell
        c.output_size, c.hidden_size = cell.input_size, cell.hidden_size
        c.mlp_hidden, c.feature_size = self.offset_predictor.hidden_size, self.feature_size
        c.rnn_type = N.LSTM if self.rnn_cell.mode == "LSTM" else N.GRU
        c.feedback = self._feedback() if feedback is None else feedback
        if self.embed_speaker is not None:
            c.num_speakers, c.speaker_dim = self.embed_speaker.num_embeddings, self.embed_speaker.embedding_dim
        return c

    def _param_list(self):
        out = []
        if self.embed_speaker is not None:
            out.append(self.embed_speaker.weight)
        out += [self.feature2hidden.weight, self.feature2hidden.bias]
        out += list(self.offset_predictor.weights())
        for m in self.emission_sampler.to_parameters.mlps:
            out += list(m.weights())
        cell = self.rnn_cell.cell
        out += [cell.weight_ih, cell.weight_hh, cell.bias_ih, cell.bias_hh]
        return out

    def _dparams(self, tensors=None):
        t = self._param_list() if tensors is None else tensors
        st = N.DecoderParams()
        i = 0
        if self.embed_speaker is not None:
            st.embed_speaker = None if t[0] is None else t[0].data_ptr()
            i = 1
        p = [None if x is None else x.data_ptr() for x in t[i:]]
        st.f2h_w, st.f2h_b = p[0], p[1]
        for name, k in (("offset", 2), ("mu", 6), ("lv", 10)):
            m = getattr(st, name)
            m.w1, m.b1, m.w2, m.b2 = p[k:k + 4]
        st.cell.w_ih, st.cell.w_hh, st.cell.b_ih, st.cell.b_hh = p[14:18]
        return st

    def workspace_bytes(self, T, L, B):
        return N.lib().abcd_decoder_workspace_bytes(self._dcfg(1), T, L, B)

    def _cfg_list(self, feedback=None):
        c = self._dcfg(feedback)
        return [c.output_size, c.hidden_size, c.mlp_hidden, c.feature_size, c.rnn_type, c.feedback, c.num_speakers,
                c.speaker_dim]

    # -- reference API --
    def forward(self, features, lengths=None, batch_sizes=None, speaker=None, ground_truth_out=None,
                ground_truth_offset=None):
        assert (lengths is not None) or (batch_sizes is not None), "Either lengths or batch_sizes must be given."
        if lengths is not None:
            batch_sizes = self._length_to_batch_sizes(lengths)
        if not torch.is_tensor(batch_sizes):
            batch_sizes = torch.tensor([int(b) for b in batch_sizes], dtype=torch.int64)
        F = self.rnn_cell.cell.input_size
        eps, seed, offset, xmask = _noise.decoder_noise(batch_sizes, F, self._input_dropout_p(), features.device)
        gt = None if ground_truth_out is None else _f32c(ground_truth_out)
        gt_off = None if ground_truth_offset is None else _f32c(ground_truth_offset)
        spk = speaker if self.embed_speaker is not None else None
        mp = _module_pad(self, "decoder")
        features = _f32c(features)
        params, cfg = self._param_list(), self._cfg_list()
        if mp is not None:  # a size not a multiple of 16: the zero-padded twin (padding.py)
            mp.twin.train(self.training)
            features, params, cfg = _pad.pad_cols(features, mp.dims.Ddp), mp.weights(params), mp.twin._cfg_list()
        em, off, flat, mu, lv, offl, _ws = ops.decoder(features, batch_sizes, spk, gt, gt_off, eps,
                                                       ops._i64(seed), ops._i64(offset), xmask, params, cfg)
        return (em if gt is not None else None), (off if gt_off is not None else None), flat, (mu, lv), offl

    def _length_to_batch_sizes(self, lengths):
        lengths = torch.as_tensor(lengths).cpu()
        return torch.tensor([int((lengths > t).sum()) for t in range(int(lengths.max()))], dtype=torch.int64)

    def pack_init_parameters(self):
        parameters = {"output_size": self.rnn_cell.cell.input_size, "rnn_hidden_size": self.rnn_cell.cell.hidden_size,
                      "mlp_hidden_size": self.offset_predictor.hidden_size, "feature_size": self.feature_size,
                      "emission_distr_name": self.emission_sampler.distribution_name,
                      "rnn_type": self.rnn_cell.mode, "rnn_layers": 1, "input_dropout": self.rnn_cell.drop.p,
                      "bidirectional": self.bidirectional}
        if self.embed_speaker is not None:
            parameters["num_speakers"] = self.embed_speaker.num_embeddings
            parameters["speaker_embed_dim"] = self.embed_speaker.embedding_dim
        return parameters
