"""ctypes binding of the C ABI in ``include/abcd_hip.h`` (``libabcd_hip.so``).

The library is built in-tree (``seq2seq_abcd-vae_amd/libabcd_hip.so``) by
``__graft_entry__.build()`` / ``make -C seq2seq_abcd-vae_amd/csrc``.  There is
no fallback: if the library (or a GPU) is missing, every compute call raises.

torch is imported first on purpose: libabcd_hip.so needs libamdhip64.so.7 and
must bind to the HIP runtime torch already loaded, so that torch's streams and
device pointers are valid for our kernels.
"""
import ctypes
import os

import torch

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("ABCD_HIP_LIB", os.path.join(PKG_DIR, "libabcd_hip.so"))

c_int, c_long, c_float, c_double, c_void_p, c_size_t, c_uint64 = (
    ctypes.c_int, ctypes.c_long, ctypes.c_float, ctypes.c_double, ctypes.c_void_p, ctypes.c_size_t,
    ctypes.c_uint64)

ABCD_EINVAL = 1000
ABCD_MAX_LAYERS = 4
LSTM, GRU = 0, 1
SAMPLE_SOFTMAX, SAMPLE_GUMBEL = 0, 1


class RnnW(ctypes.Structure):
    _fields_ = [("w_ih", c_void_p), ("w_hh", c_void_p), ("b_ih", c_void_p), ("b_hh", c_void_p)]


class MlpW(ctypes.Structure):
    _fields_ = [("w1", c_void_p), ("b1", c_void_p), ("w2", c_void_p), ("b2", c_void_p)]


class Packed(ctypes.Structure):
    _fields_ = [("data", c_void_p), ("batch_sizes", c_void_p), ("T", c_int), ("L", c_int), ("B", c_int),
                ("F", c_int)]


class EncoderCfg(ctypes.Structure):
    _fields_ = [("input_size", c_int), ("hidden_size", c_int), ("rnn_type", c_int), ("layers", c_int),
                ("bidirectional", c_int)]


class EncoderParams(ctypes.Structure):
    _fields_ = [("w", (RnnW * 2) * ABCD_MAX_LAYERS)]


class SamplerCfg(ctypes.Structure):
    _fields_ = [("input_size", c_int), ("mlp_hidden", c_int), ("num_categories", c_int),
                ("feature_dim", c_int), ("plain", c_int), ("valid_categories", c_int), ("valid_feature_dim", c_int)]


class SamplerParams(ctypes.Structure):
    _fields_ = [("mlp", MlpW * 2), ("codebook", c_void_p), ("posterior_shape_logits", c_void_p),
                ("prior_concentration", c_float)]


class SamplerGrads(ctypes.Structure):
    _fields_ = [("mlp", MlpW * 2), ("codebook", c_void_p), ("posterior_shape_logits", c_void_p)]


class DecoderCfg(ctypes.Structure):
    _fields_ = [("output_size", c_int), ("hidden_size", c_int), ("mlp_hidden", c_int), ("feature_size", c_int),
                ("rnn_type", c_int), ("feedback", c_int), ("num_speakers", c_int), ("speaker_dim", c_int)]


class DecoderParams(ctypes.Structure):
    _fields_ = [("embed_speaker", c_void_p), ("f2h_w", c_void_p), ("f2h_b", c_void_p), ("offset", MlpW),
                ("mu", MlpW), ("lv", MlpW), ("cell", RnnW)]


EncoderGrads = EncoderParams
DecoderGrads = DecoderParams

_P = ctypes.POINTER
_SIGS = {
    "abcd_version": (ctypes.c_char_p, []),
    "abcd_encoder_out_size": (c_int, [_P(EncoderCfg)]),
    "abcd_encoder_workspace_bytes": (c_size_t, [_P(EncoderCfg), c_int, c_int, c_int]),
    "abcd_encoder_forward": (c_int, [_P(EncoderCfg), _P(EncoderParams), _P(Packed), c_void_p, c_void_p, c_size_t,
                                     c_void_p]),
    "abcd_encoder_backward": (c_int, [_P(EncoderCfg), _P(EncoderParams), _P(Packed), c_void_p, _P(EncoderGrads),
                                      c_void_p, c_size_t, c_void_p]),
    "abcd_encoder_backward_overlap": (c_int, [_P(EncoderCfg), _P(EncoderParams), _P(Packed), c_void_p,
                                              _P(EncoderGrads), c_void_p, c_size_t, c_void_p, c_void_p]),
    "abcd_encoder_forward_dropout": (c_int, [_P(EncoderCfg), _P(EncoderParams), _P(Packed), c_void_p, c_void_p,
                                             c_void_p, c_size_t, c_void_p]),
    "abcd_encoder_backward_dropout": (c_int, [_P(EncoderCfg), _P(EncoderParams), _P(Packed), c_void_p, c_void_p,
                                              _P(EncoderGrads), c_void_p, c_size_t, c_void_p, c_void_p]),
    "abcd_sampler_workspace_bytes": (c_size_t, [_P(SamplerCfg), c_int]),
    "abcd_sampler_forward": (c_int, [_P(SamplerCfg), _P(SamplerParams), c_void_p, c_int, c_void_p, c_void_p,
                                     c_size_t, c_void_p]),
    "abcd_sampler_sample": (c_int, [_P(SamplerCfg), _P(SamplerParams), c_void_p, c_int, c_int, c_float, c_void_p,
                                    c_uint64, c_uint64, c_void_p, c_void_p, c_size_t, c_void_p]),
    "abcd_sampler_kl": (c_int, [_P(SamplerCfg), _P(SamplerParams), c_void_p, c_int, c_double, c_void_p, c_void_p,
                                c_size_t, c_void_p]),
    "abcd_sampler_prior": (c_int, [_P(SamplerCfg), _P(SamplerParams), c_int, c_double, c_void_p, c_size_t, c_void_p]),
    "abcd_sampler_forward_fused": (c_int, [_P(SamplerCfg), _P(SamplerParams), c_void_p, c_int, c_int, c_float,
                                           c_void_p, c_uint64, c_uint64, c_double, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_size_t, c_void_p]),
    "abcd_sampler_backward": (c_int, [_P(SamplerCfg), _P(SamplerParams), c_void_p, c_int, c_int, c_float, c_double,
                                      c_void_p, c_void_p, c_void_p, _P(SamplerGrads), c_void_p, c_size_t, c_void_p]),
    "abcd_sampler_backward_split": (c_int, [_P(SamplerCfg), _P(SamplerParams), c_void_p, c_int, c_int, c_float,
                                            c_double, c_void_p, c_void_p, c_void_p, _P(SamplerGrads), c_void_p,
                                            c_size_t, c_void_p, c_void_p]),
    "abcd_sampler_backward_params": (c_int, [_P(SamplerCfg), _P(SamplerParams), c_void_p, c_int, _P(SamplerGrads),
                                             c_void_p, c_size_t, c_void_p, c_void_p]),
    "abcd_sampler_sample_backward": (c_int, [_P(SamplerCfg), _P(SamplerParams), c_int, c_int, c_float, c_void_p,
                                             c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "abcd_sampler_kl_backward": (c_int, [_P(SamplerCfg), _P(SamplerParams), c_int, c_double, c_void_p, c_int,
                                         c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "abcd_sampler_forward_backward": (c_int, [_P(SamplerCfg), _P(SamplerParams), c_void_p, c_int, c_void_p,
                                              c_void_p, _P(SamplerGrads), c_int, c_void_p, c_size_t, c_void_p]),
    "abcd_perplexities": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "abcd_shape_perplexity": (c_int, [c_void_p, c_int, c_void_p, c_void_p]),
    "abcd_decoder_workspace_bytes": (c_size_t, [_P(DecoderCfg), c_int, c_int, c_int]),
    "abcd_decoder_forward": (c_int, [_P(DecoderCfg), _P(DecoderParams), _P(Packed), c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_size_t, c_void_p]),
    "abcd_decoder_backward": (c_int, [_P(DecoderCfg), _P(DecoderParams), _P(Packed), c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, _P(DecoderGrads), c_void_p, c_size_t, c_void_p]),
    "abcd_decoder_backward_overlap": (c_int, [_P(DecoderCfg), _P(DecoderParams), _P(Packed), c_void_p, c_void_p,
                                              c_void_p, c_void_p, c_void_p, c_void_p, _P(DecoderGrads), c_void_p,
                                              c_size_t, c_void_p, c_void_p]),
    "abcd_decoder_forward_dropout": (c_int, [_P(DecoderCfg), _P(DecoderParams), _P(Packed), c_void_p, c_void_p,
                                             c_void_p, c_void_p, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p,
                                             c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "abcd_decoder_forward_split": (c_int, [_P(DecoderCfg), _P(DecoderParams), _P(Packed), c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p]),
    "abcd_decoder_backward_dropout": (c_int, [_P(DecoderCfg), _P(DecoderParams), _P(Packed), c_void_p, c_void_p,
                                              c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, _P(DecoderGrads),
                                              c_void_p, c_size_t, c_void_p, c_void_p]),
    "abcd_decoder_backward_params": (c_int, [_P(DecoderCfg), _P(DecoderParams), _P(Packed), c_void_p, c_void_p,
                                             c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, _P(DecoderGrads),
                                             c_void_p, c_size_t, c_void_p, c_void_p]),
    "abcd_stft_frames": (c_int, [ctypes.c_longlong, c_int, c_int, c_int]),
    "abcd_featurize_workspace_bytes": (c_size_t, [c_int, c_int]),
    "abcd_featurize_packed": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_float,
                                      c_float, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_size_t,
                                      c_void_p]),
    "abcd_optim_workspace_bytes": (c_size_t, [c_long]),
    "abcd_grad_norm": (c_int, [c_void_p, c_long, c_void_p, c_void_p, c_size_t, c_void_p]),
    "abcd_clip_sgd": (c_int, [c_void_p, c_void_p, c_void_p, c_long, c_float, c_float, c_float, c_int, c_void_p,
                              c_void_p, c_size_t, c_void_p]),
    "abcd_total_loss": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "abcd_gemm_nt": (c_int, [c_int, c_int, c_int, c_void_p, c_long, c_void_p, c_long, c_void_p, c_long, c_void_p,
                             c_void_p, c_size_t, c_void_p]),
    "abcd_lstm_wgrad_workspace_bytes": (ctypes.c_size_t, [c_int, c_int, c_int, c_int]),
    "abcd_lstm_wgrad": (c_int, [c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_long, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_void_p, ctypes.c_size_t, c_void_p]),
    "abcd_gemm_tn": (c_int, [c_int, c_int, c_int, c_void_p, c_long, c_void_p, c_long, c_void_p, c_long, c_void_p,
                             c_size_t, c_void_p]),
    "abcd_linear": (c_int, [c_int, c_int, c_int, c_void_p, c_long, c_void_p, c_long, c_void_p, c_int, c_void_p,
                            c_long, c_void_p, c_size_t, c_void_p]),
    "abcd_linear_backward_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "abcd_linear_backward": (c_int, [c_int, c_int, c_int, c_void_p, c_long, c_void_p, c_long, c_void_p, c_long,
                                     c_int, c_void_p, c_long, c_void_p, c_long, c_void_p, c_void_p, c_void_p,
                                     c_size_t, c_void_p]),
    "abcd_timing_enable": (None, [c_int]),
    "abcd_timing_reset": (None, []),
    "abcd_timing_read": (c_int, [ctypes.POINTER(c_double)]),
    "abcd_timing_read_kernel": (c_int, [c_int, ctypes.POINTER(c_double)]),
    "abcd_dispatch_name": (ctypes.c_char_p, [c_int]),
    "abcd_dispatch_count": (c_long, [c_int]),
    "abcd_dispatch_reset": (None, []),
    "abcd_debug_persist_prof": (None, [c_void_p, c_int]),
    "abcd_side_gate_enable": (None, [c_int]),
    "abcd_debug_xcc_map": (c_int, [c_void_p, c_int, c_void_p]),
    "abcd_fill_normal": (c_int, [c_void_p, c_long, c_uint64, c_uint64, c_void_p]),
    "abcd_fill_dropout": (c_int, [c_void_p, c_long, c_float, c_uint64, c_uint64, c_void_p]),
    "abcd_device_status": (c_int, []),
    "abcd_step_status": (c_int, [c_void_p, c_void_p]),
}
EXPORTED = sorted(_SIGS)

_lib = None


def lib():
    """The loaded libabcd_hip.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.isfile(LIB_PATH):
            raise RuntimeError(f"libabcd_hip.so not found at {LIB_PATH}: run __graft_entry__.build() "
                               "(make -C seq2seq_abcd-vae_amd/csrc). There is no CPU fallback.")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


class HipError(RuntimeError):
    pass


class PersistTimeout(HipError):
    """A persistent recurrent kernel's hand-off wait timed out: the grid was
    not co-resident and the step's results are invalid."""


def raise_on_status(status, where):
    if status:
        raise PersistTimeout(f"{where}: a persistent recurrent kernel timed out waiting for its group "
                             f"(status {int(status)}); the results of that step are invalid")


def source_hash():
    """sha256 (first 16 hex digits) of the sources libabcd_hip.so is built
    from, concatenated in the Makefile's sorted HASHED order; abcd_version()
    ends with the same digits when the loaded library was built from this tree."""
    import hashlib
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
    names = ["abcd_gemm.hip", "abcd_rnn.hip", "abcd_persist.hip", "abcd_sampler.hip", "abcd_optim.hip",
             "abcd_feat.hip", "abcd_common.h", "abcd_internal.h", "abcd_persist.h", "abcd_x6.h",
             "../../include/abcd_hip.h"]
    h = hashlib.sha256()
    for n in sorted(names):
        with open(os.path.join(csrc, n), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def library_hash():
    """The source hash abcd_version() of the loaded library reports."""
    return lib().abcd_version().decode().rsplit(" ", 1)[-1]


class _OpStatus:
    """Bounded-latency timeout check for the op surface (ops.encoder /
    ops.decoder and their backwards, encode.py): after each persistent
    launch the device's timeout word is folded into a device slot
    (abcd_step_status) and copied without blocking into pinned host memory;
    the next probe reads the previous copy once its event has completed and
    raises PersistTimeout on a non-zero value.  sync() is the blocking form
    for the end of a batch of work (encode.py).

    A probe folds (and so clears) the device's per-launch timeout word, which
    FusedStep's STATUS slot also folds: use the op surface's probes and
    FusedStep in separate processes (the trainer uses FusedStep only, the
    encode CLIs the op surface only), or a timeout may be reported by one of
    them only."""

    def __init__(self):
        self.host = None
        self.event = None
        self.where = None

    def _read(self, block):
        if self.event is None or not (block or self.event.query()):
            return
        self.event.synchronize()
        self.event = None
        raise_on_status(float(self.host[0]), self.where)

    def probe(self, device, where):
        try:
            self._read(False)
        except PersistTimeout:
            lib().abcd_device_status()  # reported once: clear the sticky word as sync() does
            raise
        if self.event is not None:  # the previous copy is still in flight; the word keeps any new timeout
            return
        if self.host is None:
            self.host = torch.zeros(1, pin_memory=True)
        slot = torch.empty(1, device=device)
        check(lib().abcd_step_status(ptr(slot), stream()), "status probe")
        self.host.copy_(slot, non_blocking=True)
        self.event = torch.cuda.Event()
        self.event.record()
        self.where = where

    def sync(self, where):
        """Blocking check: raises PersistTimeout if any persistent launch
        timed out since the last check; always reads AND clears the device's
        status words (abcd_device_status), so a reported timeout is not
        reported again by the next check."""
        try:
            self._read(True)
        except PersistTimeout:
            lib().abcd_device_status()
            raise
        raise_on_status(lib().abcd_device_status(), where)


op_status = _OpStatus()


def check(rc, what):
    if rc != 0:
        if rc == ABCD_EINVAL:
            raise HipError(f"{what}: invalid or unsupported arguments (ABCD_EINVAL)")
        raise HipError(f"{what}: HIP error {rc}")


def require_gpu(t):
    if not (torch.is_tensor(t) and t.is_cuda):
        raise RuntimeError("the ABCD-VAE HIP path runs on an MI355X GPU only; got a tensor on "
                           f"{getattr(t, 'device', None)} (no CPU fallback)")


def ptr(t):
    return None if t is None else c_void_p(t.data_ptr())


def stream():
    return c_void_p(torch.cuda.current_stream().cuda_stream)


SAMPLE_PRIOR_READY = 0x100  # abcd_hip.h ABCD_SAMPLE_PRIOR_READY
DEFER_PARAMS = c_void_p(2 ** 64 - 1)  # abcd_hip.h ABCD_DEFER_PARAMS ((void*)-1)


def workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


ENC_FWD, ENC_BWD, DEC_FWD, DEC_BWD, SAMP_FWD, SAMP_BWD, ENC_WGRAD = 1, 2, 3, 4, 5, 6, 7


def dispatch():
    """{role: (kernel name of its last launch, launches since reset)}"""
    L = lib()
    return {r: (L.abcd_dispatch_name(k).decode(), int(L.abcd_dispatch_count(k)))
            for r, k in (("enc_fwd", ENC_FWD), ("enc_bwd", ENC_BWD), ("dec_fwd", DEC_FWD), ("dec_bwd", DEC_BWD),
                                ("samp_fwd", SAMP_FWD), ("samp_bwd", SAMP_BWD), ("enc_wgrad", ENC_WGRAD))}


def ptr_array(tensors):
    """HOST array of device pointers (None entries -> NULL), or None if all None."""
    if tensors is None or all(t is None for t in tensors):
        return None
    arr = (c_void_p * len(tensors))(*[None if t is None else t.data_ptr() for t in tensors])
    return arr
