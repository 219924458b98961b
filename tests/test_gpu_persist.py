"""Persistent recurrent kernels (abcd_persist.hip): the whole encoder time loop
in one launch per layer, workgroups handing the recurrent state to each other
inside the launch.

* against torch.nn.LSTM/GRU in float64 on the CPU (the op the reference's
  encoder is, ABCD-VAE/modules/model.py:53,60-66) on ragged packed batches
  whose row-tile count is not a multiple of 8 (the non-XCD group mapping);
* against the per-step kernels (ABCD_PERSIST=0) at the benchmark size
  (H=256, batch 512, T=200: 16 groups of 16 workgroups, XCD-aware mapping);
* every run ends with abcd_device_status() == 0 (no hand-off wait timed out).
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _enc(F, H, rnn, layers, bidir, seed):
    from modules import model as M
    torch.manual_seed(seed)
    return M.RNN_Variational_Encoder(F, H, rnn_type=rnn, rnn_layers=layers, bidirectional=bidir).cuda()


def _batch(B, Tmax, F, seed):
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(1, Tmax + 1, (B,), generator=g)
    lens[0] = Tmax
    lens = lens.sort(descending=True).values
    seqs = [torch.randn(int(n), F, generator=g) for n in lens]
    return torch.nn.utils.rnn.pack_sequence(seqs)


def _run(enc, packed, dout, persist):
    from modules import _native as Nn
    old = os.environ.get("ABCD_PERSIST")
    os.environ["ABCD_PERSIST"] = "1" if persist else "0"
    try:
        data = packed.data.cuda()
        for p in enc.parameters():
            p.grad = None
        out = enc(torch.nn.utils.rnn.PackedSequence(data, packed.batch_sizes))
        (out * dout).sum().backward()
        torch.cuda.synchronize()
        assert Nn.lib().abcd_device_status() == 0
        return out.detach().cpu().double(), {n: p.grad.detach().cpu().double() for n, p in enc.rnn.named_parameters()}
    finally:
        if old is None:
            os.environ.pop("ABCD_PERSIST", None)
        else:
            os.environ["ABCD_PERSIST"] = old


def _torch_ref(enc, packed, dout):
    rnn = enc.rnn
    cls = torch.nn.LSTM if rnn.mode == "LSTM" else torch.nn.GRU
    ref = cls(rnn.input_size, rnn.hidden_size, rnn.num_layers, bidirectional=rnn.bidirectional,
              batch_first=True).double()
    with torch.no_grad():
        for n, p in ref.named_parameters():
            p.copy_(getattr(rnn, n).detach().cpu().double())
    _, hn = ref(torch.nn.utils.rnn.PackedSequence(packed.data.double(), packed.batch_sizes))
    if rnn.mode == "LSTM":
        hn = torch.cat(hn, dim=-1)
    out = hn.transpose(0, 1).contiguous().view(hn.shape[1], -1)
    (out * dout.cpu().double()).sum().backward()
    return out.detach(), {n: p.grad for n, p in ref.named_parameters()}


def _rel(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


@pytest.mark.parametrize("rnn,layers,bidir", [("LSTM", 1, True), ("GRU", 1, True), ("LSTM", 2, True),
                                              ("LSTM", 1, False), ("GRU", 2, False)])
def test_persistent_encoder_vs_torch_f64(rnn, layers, bidir):
    F, H, B, Tmax = 33, 64, 150, 40
    enc = _enc(F, H, rnn, layers, bidir, seed=7)
    packed = _batch(B, Tmax, F, seed=11)
    dout = torch.randn(B, enc.hidden_size_total, device="cuda")
    out, grads = _run(enc, packed, dout, persist=True)
    rout, rgrads = _torch_ref(enc, packed, dout)
    assert _rel(out, rout) < 1e-5
    for n, g in rgrads.items():
        assert _rel(grads[n], g) < 1e-4, n


@pytest.mark.parametrize("rnn", ["LSTM", "GRU"])
def test_persistent_encoder_vs_stepwise_bench_size(rnn):
    F, H, B, Tmax = 129, 256, 512, 200
    enc = _enc(F, H, rnn, 1, True, seed=3)
    packed = _batch(B, Tmax, F, seed=5)
    dout = torch.randn(B, enc.hidden_size_total, device="cuda")
    out_p, g_p = _run(enc, packed, dout, persist=True)
    out_s, g_s = _run(enc, packed, dout, persist=False)
    assert _rel(out_p, out_s) < 1e-5
    for n in g_s:
        assert _rel(g_p[n], g_s[n]) < 1e-4, n
    # repeated launches reuse the zeroed counters: identical results
    out_p2, g_p2 = _run(enc, packed, dout, persist=True)
    assert torch.equal(out_p, out_p2)
    for n in g_p:
        assert torch.equal(g_p[n], g_p2[n]), n


def _with_env(key, val, fn):
    old = os.environ.get(key)
    os.environ[key] = val
    try:
        return fn()
    finally:
        if old is None:
            os.environ.pop(key, None)
        else:
            os.environ[key] = old


@pytest.mark.parametrize("wg", ["3", "2"])
@pytest.mark.parametrize("B,Tmax", [(70, 30), (512, 200)])
def test_encoder_wgrad_wg2(B, Tmax, wg):
    """The layer-0 bi-LSTM weight gradients through gemm_wg3b (default) and
    gemm_wg2 (ABCD_WG3=0) -- one launch for both directions: [dW_ih | db |
    dW_hh] = dG^T [X | 1 | Hprev], F = 129, H = 256 -- against the split GEMM
    route (ABCD_WG2=0) and, at the small batch, against torch.nn.LSTM in
    float64 (model.py:53,60-66)."""
    from modules import _native as Nn
    F, H = 129, 256
    enc = _enc(F, H, "LSTM", 1, True, seed=5)
    packed = _batch(B, Tmax, F, seed=9)
    dout = torch.randn(B, enc.hidden_size_total, device="cuda")
    Nn.lib().abcd_dispatch_reset()
    out_n, g_n = _with_env("ABCD_WG3", "1" if wg == "3" else "0", lambda: _run(enc, packed, dout, persist=True))
    assert Nn.dispatch()["enc_wgrad"] == (f"gemm_wg{'3b' if wg == '3' else wg}<144,256> x2", 1)
    out_o, g_o = _with_env("ABCD_WG2", "0", lambda: _run(enc, packed, dout, persist=True))
    assert Nn.dispatch()["enc_wgrad"] == ("gemm split (x6s/x6t)", 2)
    assert torch.equal(out_n, out_o)
    for n in g_o:
        assert _rel(g_n[n], g_o[n]) < 1e-5, (n, _rel(g_n[n], g_o[n]))
    if B <= 128:
        _, rgrads = _torch_ref(enc, packed, dout)
        for n, g in rgrads.items():
            assert _rel(g_n[n], g) < 1e-4, (n, _rel(g_n[n], g))


def _fused_run(step, batch, persist, seed=77):
    from modules import _native as Nn, noise
    old = os.environ.get("ABCD_PERSIST")
    os.environ["ABCD_PERSIST"] = "1" if persist else "0"
    try:
        noise.set_mode("philox")
        noise.manual_seed(seed)
        step.flat.grad.zero_()
        sc, logits = step.forward_backward(batch["data"], batch["batch_sizes"], batch["is_offset"],
                                           batch["speakers"], 10000)
        torch.cuda.synchronize()
        assert Nn.lib().abcd_device_status() == 0
        return sc.detach().cpu().double().clone(), step.flat.grad.detach().cpu().double().clone()
    finally:
        if old is None:
            os.environ.pop("ABCD_PERSIST", None)
        else:
            os.environ["ABCD_PERSIST"] = old


ODD = dict(workload="odd shapes", F=33, H=48, Hm=32, D=32, K=16, rnn="LSTM", plain=False, tmin=3, tmax=30, B=100,
           N=1000, spk=0, sdim=None)


@pytest.mark.parametrize("cfg_name", ["c2", "c4", "c5", "c5gru", "odd"])
def test_fused_step_persist_vs_stepwise_bench_size(cfg_name):
    """Whole training step (encoder + sampler + decoder, forward + backward) at
    the benchmark configuration: persistent kernels vs the per-step kernels;
    c5 / c5gru: the stress configuration of BASELINE.json (K = 1024, speaker
    embedding 256, T_max = 512); "odd": K-chunk counts that are not multiples
    of the ring depth (H = 48, Fp = 48), two row tiles with a ragged one."""
    import bench
    cfg = ODD if cfg_name == "odd" else bench.CONFIGS[cfg_name]
    step = bench.build(cfg, "cuda")
    batch = bench.make_batch(cfg, 0, "cuda")
    sc_p, g_p = _fused_run(step, batch, True)
    sc_s, g_s = _fused_run(step, batch, False)
    # losses (EM, OFF, KL, LOSS) within 1e-5 relative; gradient vector within 1e-4 of its max
    for k in range(4):
        assert abs(sc_p[k] - sc_s[k]) <= 1e-5 * abs(sc_s[k]) + 1e-6, (k, sc_p[k].item(), sc_s[k].item())
    assert _rel(g_p, g_s) < 1e-4


@pytest.mark.parametrize("rnn", ["LSTM", "GRU"])
def test_decoder_input_dropout_persist_vs_stepwise(rnn):
    """Decoder input dropout 0 < p < 1 in training (RNN_Cell's nn.Dropout,
    ABCD-VAE/modules/model.py:289,297) at c2 widths: the persistent decoder
    kernels (mask applied to the fed-back sample before the hand-off, and to
    dx in the BPTT's emission epilogue) agree with the per-step kernels, and
    the mask changes the result (it is applied at all)."""
    import bench
    cfg = dict(bench.CONFIGS["c2"], rnn=rnn)
    step = bench.build(cfg, "cuda")
    batch = bench.make_batch(cfg, 0, "cuda")
    sc_0, g_0 = _fused_run(step, batch, True)
    step.decoder.rnn_cell.drop.p = 0.3
    sc_p, g_p = _fused_run(step, batch, True)
    sc_s, g_s = _fused_run(step, batch, False)
    for k in range(4):
        assert abs(sc_p[k] - sc_s[k]) <= 1e-5 * abs(sc_s[k]) + 1e-6, (k, sc_p[k].item(), sc_s[k].item())
    assert _rel(g_p, g_s) < 1e-4
    assert sc_p[0] != sc_0[0] and _rel(g_p, g_0) > 1e-3


@pytest.mark.parametrize("cfg_name", ["c2", "c5gru", "odd"])
def test_fused_decoder_init_vs_gemm(cfg_name):
    """feature2hidden formed straight into the decoder's initial state
    (dec_init_f2h, the default) against the split-K GEMM + dec_init scatter
    (ABCD_DEC_INIT_F2H=0), model.py:100,262-263: the whole training step at
    c2 (DS = 256, LSTM h / c interleave), c5gru (DS = 512 with the speaker
    embedding, GRU) and the odd shapes (DS = 32, a ragged 32-column tile)."""
    import bench
    cfg = ODD if cfg_name == "odd" else bench.CONFIGS[cfg_name]
    step = bench.build(cfg, "cuda")
    batch = bench.make_batch(cfg, 0, "cuda")
    sc_f, g_f = _with_env("ABCD_DEC_INIT_F2H", "1", lambda: _fused_run(step, batch, True))
    sc_g, g_g = _with_env("ABCD_DEC_INIT_F2H", "0", lambda: _fused_run(step, batch, True))
    for k in range(4):
        assert abs(sc_f[k] - sc_g[k]) <= 1e-5 * abs(sc_g[k]) + 1e-6, (k, sc_f[k].item(), sc_g[k].item())
    assert _rel(g_f, g_g) < 1e-4
