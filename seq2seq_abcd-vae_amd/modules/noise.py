"""Noise sources for the stochastic parts of the step (Gumbel, Gaussian).

Two modes:

* ``"philox"`` (default, production): the kernels draw Philox-4x32-10
  counter-based noise in place (``abcd_common.h``), keyed by ``(seed, offset)``;
  nothing is drawn or copied on the host.  The stream is advanced like torch's
  own CUDA Philox generator: one offset block per draw.
* ``"reference"``: the noise is drawn on the HOST from torch's global CPU
  generator, with exactly the calls, shapes and order the reference makes
  (``F.gumbel_softmax``'s ``-empty_like(logits).exponential_().log()``,
  ``model.py:604``; ``randn_like(mean)`` per decoder step, ``model.py:19``;
  the plain sampler's ``randn_like(mean)``), then uploaded.  This reproduces a
  reference CPU run's random numbers bit-for-bit and is what
  the parity tests and the toy-trajectory check use.
"""
import torch

_state = {"mode": "philox", "seed": 0x5EED1111, "offset": 0}
_replay = []  # FIFO of host tensors consumed before any other source (tests / replays)


def replay(*tensors):
    """Queue exact noise tensors (e.g. recorded from a reference run); each
    draw pops one, in call order, and checks its shape."""
    _replay.extend(tensors)


def _pop(shape, device):
    t = _replay.pop(0)
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"replayed noise has shape {tuple(t.shape)}, draw wants {tuple(shape)}")
    return t.to(device=device, dtype=torch.float32).contiguous(), 0, 0


def set_mode(mode):
    if mode not in ("philox", "reference"):
        raise ValueError(f"noise mode must be 'philox' or 'reference', not {mode!r}")
    _state["mode"] = mode


def get_mode():
    return _state["mode"]


def manual_seed(seed, rank=0):
    """Seed the Philox stream.  Under data parallelism every rank passes its
    rank: rank r > 0 gets its own key (seed xor a rank hash), so the ranks'
    shards draw independent Gumbel / decoder / dropout noise as one device
    would for the global batch; rank 0 keeps the single-device stream."""
    key = int(seed) & 0xFFFFFFFFFFFFFFFF
    if rank:
        key ^= (0x9E3779B97F4A7C15 * (int(rank) + 1)) & 0xFFFFFFFFFFFFFFFF
    _state["seed"] = key
    _state["offset"] = 0


def get_state():
    return dict(_state)


def set_state(st, rank=0):
    """Restore a state saved by get_state (rank 0's, under data parallelism);
    rank r > 0 re-derives its own key from it (manual_seed's rank hash)."""
    _state.update({k: st[k] for k in ("mode", "seed", "offset") if k in st})
    if rank and "seed" in st:
        _state["seed"] = (int(st["seed"]) ^ ((0x9E3779B97F4A7C15 * (int(rank) + 1)) & 0xFFFFFFFFFFFFFFFF))


class mode:
    """Context manager: ``with noise.mode("reference"): ...``"""

    def __init__(self, m):
        self.m = m

    def __enter__(self):
        self.prev = get_mode()
        set_mode(self.m)

    def __exit__(self, *exc):
        set_mode(self.prev)


def philox(n):
    """Reserve n counters of the Philox stream: returns (seed, offset)."""
    off = _state["offset"]
    _state["offset"] = off + ((int(n) + 3) // 4) * 4
    return _state["seed"], off


def gumbel(B, K, device, width=None):
    """(noise tensor or None, seed, offset) for a B x K Gumbel draw.  width:
    the row stride the kernel reads Philox counters with (a zero-padded model,
    modules/padding.py): host noise is returned zero-padded to it, the Philox
    reservation covers B x width counters."""
    width = K if width is None else int(width)
    if _replay:
        t, s, o = _pop((B, K), device)
        return _widen(t, width), s, o
    if _state["mode"] == "reference":
        g = -torch.empty(B, K).exponential_().log()
        return _widen(g.to(device, non_blocking=True), width), 0, 0
    s, o = philox(B * width)
    return None, s, o


def normal(B, f, device, width=None):
    """(noise tensor or None, seed, offset) for a B x f standard normal draw (width: as gumbel)."""
    width = f if width is None else int(width)
    if _replay:
        t, s, o = _pop((B, f), device)
        return _widen(t, width), s, o
    if _state["mode"] == "reference":
        return _widen(torch.randn(B, f).to(device, non_blocking=True), width), 0, 0
    s, o = philox(B * width)
    return None, s, o


def _widen(t, width):
    if t.shape[-1] == width:
        return t
    return torch.nn.functional.pad(t, (0, width - t.shape[-1]))


def decoder_eps(batch_sizes, F, device):
    """Per-step ``randn(bs_t, F)`` in packed order (reference) or a Philox block."""
    L = int(sum(int(b) for b in batch_sizes))
    if _replay:
        return _pop((L, F), device)
    if _state["mode"] == "reference":
        eps = torch.cat([torch.randn(int(bs), F) for bs in batch_sizes], 0)
        return eps.to(device, non_blocking=True), 0, 0
    s, o = philox(L * F)
    return None, s, o


def decoder_noise(batch_sizes, F, p, device):
    """Noise of one training-mode decoder pass with input dropout p:
    (eps, seed, offset, xmask).  0 < p < 1 adds the RNN_Cell dropout noise of
    every step's cell input (model.py:297, ``nn.Dropout(p)`` on
    ``batched_input[:bs_t]``), an L x F tensor in packed order.  In reference
    mode the two draws interleave per step exactly as the reference loop makes
    them (dropout of step t's input, then the sampler's ``randn(bs_t, F)``,
    model.py:186-188, 19); otherwise eps is a Philox block and the mask comes
    from abcd_fill_dropout.  Replays pop eps then the mask."""
    if not (0.0 < p < 1.0):
        return decoder_eps(batch_sizes, F, device) + (None,)
    L = int(sum(int(b) for b in batch_sizes))
    if _replay:
        eps = _pop((L, F), device)
        return eps + (_pop((L, F), device)[0],)
    if _state["mode"] == "reference":
        masks, eps = [], []
        for bs in batch_sizes:
            masks.append(torch.empty(int(bs), F).bernoulli_(1 - p).div_(1 - p))
            eps.append(torch.randn(int(bs), F))
        return (torch.cat(eps, 0).to(device, non_blocking=True), 0, 0,
                torch.cat(masks, 0).to(device, non_blocking=True))
    eps, s, o = decoder_eps(batch_sizes, F, device)
    return eps, s, o, dropout_noise((L, F), p, device)


def dropout_noise(shape, p, device):
    """Training-mode dropout noise bernoulli(1 - p) / (1 - p) of `shape`
    (ATen's _dropout_impl: ``empty_like(x).bernoulli_(1 - p).div_(1 - p)``):
    drawn on the host from torch's CPU generator in reference mode (bit-exact
    with a reference CPU run), from the Philox stream by abcd_fill_dropout
    otherwise.  Returns a device tensor."""
    if _state["mode"] == "reference":
        return torch.empty(*shape).bernoulli_(1 - p).div_(1 - p).to(device, non_blocking=True)
    from . import _native as N
    out = torch.empty(*shape, device=device)
    n = out.numel()
    s, o = philox(n)
    N.check(N.lib().abcd_fill_dropout(N.ptr(out), n, float(p), s, o, N.stream()), "dropout noise")
    return out
