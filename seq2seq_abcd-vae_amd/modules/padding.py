# coding: utf-8
"""Any model size on the 16-multiple kernels: the zero-padded model.

The reference accepts every ``-K``, ``-f``, ``--encoder_rnn_hidden_size``,
``--decoder_rnn_hidden_size``, ``--mlp_hidden_size`` and ``--speaker_embed_dim``
(``ABCD-VAE/learning.py:371-376``; ``model.py:53,91,542``).  The kernels tile
those dimensions by 16.  A model whose sizes are not multiples of 16 runs as
its ZERO-PADDED twin: every size rounded up to 16, each real weight embedded
at its unit / gate / block position, every padding weight 0.

Why that is exact:

* LSTM padding unit: gates = 0 + 0, so i = f = o = 1/2, g = tanh 0 = 0; with
  c_0 = 0 the cell stays c = 0 and h = 0 at every step.  GRU: n = tanh 0 = 0,
  h' = z h = 0.  Their recurrent columns are 0 as well, so they never feed a
  real unit, and every gradient reaching them is 0 (the consumers' columns
  are 0).
* MLP padding unit: tanh(0) = 0 into a zero column.  Codebook padding
  dimension: U = 0 and a zero codebook row.  Padding input columns (encoder
  output, features, speaker embedding) meet zero weight columns.
* Padding categories are the one place the real size is visible: a zero
  logit would still take softmax mass, and the Dirichlet prior sums over K.
  The sampler kernels mask them (``abcd_sampler_cfg.valid_categories``) and
  scale the logits by 1 / sqrt(real D) (``valid_feature_dim``).

So values and gradients at the real positions are the real model's (up to
fp32 summation order).  Two users:

* ``PadPlan`` -- the fused training step (``engine.FusedStep``): twin modules
  of the whole model (the encoder's output blocks ``[h_f, c_f, h_b, c_b]``
  widened block by block, the sampler's input columns following them) and
  the index map real flat parameters -> padded flat parameters; the step
  embeds the parameters (one ``index_copy``) and gathers the gradients (one
  ``index_select``), while the all-reduce, clip + SGD and checkpoints stay on
  the real parameters.
* ``ModulePad`` -- the nn.Module surface (``model.py``): each module pads its
  own sizes with differentiable embeddings per call, the tensors between
  modules keep their real sizes.
"""
from types import SimpleNamespace

import torch


def up16(n):
    return -(-int(n) // 16) * 16


def prefix(n):
    return torch.arange(int(n))


def blocks(nb, n, npad):
    """nb consecutive blocks of n real entries, each at the start of a block of npad."""
    return (torch.arange(int(nb))[:, None] * int(npad) + torch.arange(int(n))[None, :]).reshape(-1)


def concat_blocks(sizes, pads):
    """Blocks of different widths: real block i (sizes[i]) at the start of padded block i (pads[i])."""
    out, base = [], 0
    for n, p in zip(sizes, pads):
        out.append(base + torch.arange(int(n)))
        base += int(p)
    return torch.cat(out)


# ----------------------------------------------------------------------------
# sizes of each module (real and padded)
# ----------------------------------------------------------------------------
def encoder_dims(enc):
    r = enc.rnn
    d = SimpleNamespace(F=r.input_size, H=r.hidden_size, Hp=up16(r.hidden_size), G=4 if r.mode == "LSTM" else 3,
                        dirs=2 if r.bidirectional else 1, nblk=enc.hidden_size_total // r.hidden_size)
    d.active = d.H != d.Hp
    d.out_cols = blocks(d.nblk, d.H, d.Hp)  # real columns of the padded last_hidden
    return d


def sampler_dims(samp, in_cols=None, in_width=None):
    """in_cols / in_width: where the sampler's input columns sit in its padded
    input (fused step: the encoder's output blocks); default: a prefix of up16(E)."""
    from .model import ABCDSampler
    abcd = isinstance(samp, ABCDSampler)
    m = samp.to_code_like if abcd else samp.to_parameters
    E = m.input_size
    d = SimpleNamespace(abcd=abcd, E=E, Hm=m.hidden_size, D=m.output_size, K=samp.num_categories if abcd else 0)
    d.in_cols = prefix(E) if in_cols is None else in_cols
    d.Ep = up16(E) if in_width is None else int(in_width)
    d.Hmp, d.Dp, d.Kp = up16(d.Hm), up16(d.D), (up16(d.K) if abcd else 0)
    d.active = (d.Ep, d.Hmp, d.Dp, d.Kp) != (E, d.Hm, d.D, d.K)
    return d


def decoder_dims(dec):
    cell = dec.rnn_cell.cell
    d = SimpleNamespace(F=cell.input_size, Hd=cell.hidden_size, Gd=4 if dec.rnn_cell.mode == "LSTM" else 3,
                        lstm=dec.rnn_cell.mode == "LSTM", Hmd=dec.offset_predictor.hidden_size,
                        Dd=dec.feature_size, S=dec.embed_speaker.embedding_dim if dec.embed_speaker is not None else 0,
                        nspk=dec.embed_speaker.num_embeddings if dec.embed_speaker is not None else 0)
    d.Hdp, d.Hmdp, d.Ddp, d.Sp = up16(d.Hd), up16(d.Hmd), up16(d.Dd), (up16(d.S) if d.S else 0)
    d.active = (d.Hdp, d.Hmdp, d.Ddp, d.Sp) != (d.Hd, d.Hmd, d.Dd, d.S)
    return d


# ----------------------------------------------------------------------------
# per-parameter layouts: (rows, cols) of the real entries in the padded tensor
# ----------------------------------------------------------------------------
def encoder_layout(d, name):
    """``rnn.<name>`` of RNN_Variational_Encoder: gate blocks of H in G * Hp rows."""
    gate = blocks(d.G, d.H, d.Hp)
    kind, rest = name.split("_l")
    layer = int(rest.split("_")[0])
    if kind == "weight_ih":
        return gate, (prefix(d.F) if layer == 0 else blocks(d.dirs, d.H, d.Hp))
    if kind == "weight_hh":
        return gate, prefix(d.H)
    return gate, None


def sampler_layout(d, name):
    if name == "posterior_shape_logits":
        return prefix(d.K), None
    if name == "codebook":
        return prefix(d.D), prefix(d.K)
    layer, kind = name.split(".")[-2:]  # <mlp>.whole_network.{0,2}.{weight,bias}
    if layer == "0":
        return (prefix(d.Hm), d.in_cols) if kind == "weight" else (prefix(d.Hm), None)
    return (prefix(d.D), prefix(d.Hm)) if kind == "weight" else (prefix(d.D), None)


def decoder_layout(d, name):
    htot = 2 * d.Hd if d.lstm else d.Hd  # feature2hidden rows, (h, c) interleaved per unit: a prefix
    if name == "embed_speaker.weight":
        return prefix(d.nspk), prefix(d.S)
    if name == "feature2hidden.weight":
        return prefix(htot), (concat_blocks([d.Dd, d.S], [d.Ddp, d.Sp]) if d.S else prefix(d.Dd))
    if name == "feature2hidden.bias":
        return prefix(htot), None
    if name.startswith("rnn_cell.cell."):
        kind = name.split(".")[-1]
        gate = blocks(d.Gd, d.Hd, d.Hdp)
        if kind == "weight_ih":
            return gate, prefix(d.F)
        if kind == "weight_hh":
            return gate, prefix(d.Hd)
        return gate, None
    layer, kind = name.split(".")[-2:]  # offset_predictor / emission MLPs: Hd -> Hmd -> (1 | F)
    out = 1 if name.startswith("offset_predictor") else d.F
    if layer == "0":
        return (prefix(d.Hmd), prefix(d.Hd)) if kind == "weight" else (prefix(d.Hmd), None)
    return (prefix(out), prefix(d.Hmd)) if kind == "weight" else (prefix(out), None)


def flat_index(rows, cols, padded_shape):
    """Flat positions in a tensor of padded_shape of the real entries (row-major)."""
    if cols is None:
        return rows.clone()
    return (rows[:, None] * int(padded_shape[1]) + cols[None, :]).reshape(-1)


def embed(t, rows, cols, padded_shape):
    """Differentiable zero-padded copy of t with t's entries at (rows, cols)."""
    out = t.new_zeros(padded_shape)
    if cols is None:
        return out.index_copy(0, rows.to(t.device), t)
    idx = flat_index(rows, cols, padded_shape).to(t.device)
    return out.reshape(-1).index_copy(0, idx, t.reshape(-1)).view(padded_shape)


# ----------------------------------------------------------------------------
# twin modules (same classes, padded sizes), built off torch's global RNG
# ----------------------------------------------------------------------------
def encoder_twin(enc, d):
    from . import model as M
    r = enc.rnn
    with torch.random.fork_rng(devices=[]):
        return M.RNN_Variational_Encoder(d.F, d.Hp, rnn_type=r.mode, rnn_layers=r.num_layers,
                                         hidden_dropout=r.dropout, bidirectional=r.bidirectional)


def sampler_twin(samp, d):
    from . import model as M
    with torch.random.fork_rng(devices=[]):
        if d.abcd:
            t = M.ABCDSampler(d.Ep, d.Hmp, d.Kp, d.Dp, prior_concentration=samp._prior_value())
        else:
            t = M.Sampler(d.Ep, d.Hmp, d.Dp, distribution_name=samp.distribution_name)
    t.valid_sizes = (d.K, d.D)
    return t


def decoder_twin(dec, d):
    from . import model as M
    with torch.random.fork_rng(devices=[]):
        return M.RNN_Variational_Decoder(d.F, d.Hdp, d.Hmdp, d.Ddp, rnn_type=dec.rnn_cell.mode,
                                         input_dropout=dec.rnn_cell.drop.p, num_speakers=d.nspk or None,
                                         speaker_embed_dim=d.Sp or None)


_LAYOUT = {"encoder": encoder_layout, "sampler": sampler_layout, "decoder": decoder_layout}


def _param_layouts(kind, real, twin, d):
    """[(real param, rows, cols, padded shape)] in the module's parameter order."""
    tp = dict(twin.named_parameters())
    out = []
    for name, p in real.named_parameters():
        key = name[len("rnn."):] if kind == "encoder" else name
        rows, cols = _LAYOUT[kind](d, key)
        assert rows.numel() * (1 if cols is None else cols.numel()) == p.numel(), name
        out.append((p, rows, cols, tuple(tp[name].shape)))
    return out


class PadPlan:
    """The fused step's padded model: twins of (encoder, sampler, decoder) and
    the index map of the real flat parameter vector (their parameters in
    order) into the twins' flat vector."""

    def __init__(self, enc, samp, dec):
        de = encoder_dims(enc)
        ds = sampler_dims(samp, in_cols=de.out_cols, in_width=de.nblk * de.Hp)
        dd = decoder_dims(dec)
        self.dims = (de, ds, dd)
        self.twins = (encoder_twin(enc, de), sampler_twin(samp, ds), decoder_twin(dec, dd))
        idx, base = [], 0
        for kind, real, twin, d in zip(("encoder", "sampler", "decoder"), (enc, samp, dec), self.twins, self.dims):
            for p, rows, cols, shp in _param_layouts(kind, real, twin, d):
                idx.append(base + flat_index(rows, cols, shp))
                base += int(torch.Size(shp).numel())
        self.index = torch.cat(idx)
        self.padded_numel = base

    @staticmethod
    def needed(enc, samp, dec):
        return encoder_dims(enc).active or sampler_dims(samp).active or decoder_dims(dec).active


class ModulePad:
    """One module's padded twin for the nn.Module surface: ``weights(ts)`` embeds
    the real tensors (in the order the module hands them to its operator)
    differentiably; ``cfg`` is the twin's operator configuration."""

    def __init__(self, kind, module):
        self.kind = kind
        d = {"encoder": encoder_dims, "sampler": sampler_dims, "decoder": decoder_dims}[kind](module)
        self.dims = d
        self.twin = {"encoder": encoder_twin, "sampler": sampler_twin, "decoder": decoder_twin}[kind](module, d)
        self._by_id = {id(p): (rows, cols, shp) for p, rows, cols, shp in _param_layouts(kind, module, self.twin, d)}
        self.cfg = self.twin._cfg_list()

    def weights(self, ts):
        out = []
        for t in ts:
            rows, cols, shp = self._by_id[id(t)]
            out.append(embed(t, rows, cols, shp))
        return out

    def weight(self, t):
        return self.weights([t])[0]


def pad_cols(t, width):
    """Zero columns appended to a 2-D tensor (inputs / noise of the padded model)."""
    if t is None or t.shape[-1] == width:
        return t
    return torch.nn.functional.pad(t, (0, width - t.shape[-1]))


def pad_col_blocks(t, nb, n, npad, fill=1.0):
    """L x nb*n -> L x nb*npad with the blocks at the starts (dropout masks: fill 1)."""
    if t is None or n == npad:
        return t
    out = t.new_full((t.shape[0], nb * npad), fill)
    out[:, blocks(nb, n, npad).to(t.device)] = t
    return out
