"""The fused sampler head (abcd_sampler_forward_fused + the fused branch of
abcd_sampler_backward_split) against the three per-method entry points it
replaces (forward / sample / kl and their backward pieces, which the
reference fixtures pin: test_gpu_parity.py, test_gpu_prod.py).

Shapes: the bench configurations' sampler (E = 4H = 1024, Hm = D = 256,
K = 128 and 1024) at B = 512 (32 full 16-row tiles) and B = 72 (a ragged last
tile), Gumbel noise given explicitly, drawn in-kernel (Philox), and the plain
softmax of pre-training.

Tolerances: forward outputs 1e-5 of the tensor's max, KL 1e-5 relative,
argmax of Y exact; gradients 1e-4 of the tensor's max (the fused kernels sum
in a different order: per-tile MFMA chains instead of split-K slabs)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ck(rc):
    from modules import _native as N
    N.check(rc, "sampler head test")


def _rel(a, b):
    return float((a - b).abs().max()) / max(float(b.abs().max()), 1e-30)


def _grads(samp, dev):
    w1, b1, w2, b2 = samp._mlps()[0].weights()
    views = {"mlp0.w1": torch.zeros_like(w1), "mlp0.b1": torch.zeros_like(b1), "mlp0.w2": torch.zeros_like(w2),
             "mlp0.b2": torch.zeros_like(b2), "codebook": torch.zeros_like(samp.codebook),
             "posterior_shape_logits": torch.zeros_like(samp.posterior_shape_logits)}
    return views, samp._sgrads(views)


@pytest.mark.parametrize("K", [128, 1024])
@pytest.mark.parametrize("B", [512, 72])
@pytest.mark.parametrize("mode", ["gumbel_noise", "gumbel_philox", "softmax"])
def test_fused_head_matches_per_method_path(K, B, mode):
    from modules import model as M, _native as N
    L = N.lib()
    dev = torch.device("cuda")
    torch.manual_seed(7 + K + B)
    E, Hm, D, NDATA = 1024, 256, 256, 10000.0
    samp = M.ABCDSampler(E, Hm, K, D).to(dev)
    with torch.no_grad():
        samp.posterior_shape_logits.normal_(0.0, 0.5)
    cfg, par = samp._scfg(), samp._sparams()
    h = torch.randn(B, E, device=dev)
    gmode = N.SAMPLE_SOFTMAX if mode == "softmax" else N.SAMPLE_GUMBEL
    tau = 0.5 if gmode == N.SAMPLE_GUMBEL else 1.0
    noise = None
    if mode == "gumbel_noise":
        noise = -torch.log(torch.distributions.Exponential(torch.ones(())).sample((B, K)).to(dev))
    seed, off = 1234, 99
    d_feats = torch.randn(B, D, device=dev) / B
    d_kl = torch.full((), 1.0 / B, device=dev)
    nbytes = L.abcd_sampler_workspace_bytes(cfg, B)
    st = N.stream()

    # per-method path: forward, sample, kl; sample / kl / forward backward pieces
    wa = N.workspace(nbytes, dev)
    la, fa, ka = torch.empty(B, K, device=dev), torch.empty(B, D, device=dev), torch.empty(1, device=dev)
    _ck(L.abcd_sampler_forward(cfg, par, N.ptr(h), B, N.ptr(la), N.ptr(wa), wa.numel(), st))
    _ck(L.abcd_sampler_sample(cfg, par, N.ptr(la), B, gmode, tau, N.ptr(noise), seed, off, N.ptr(fa), N.ptr(wa),
                                  wa.numel(), st))
    _ck(L.abcd_sampler_kl(cfg, par, N.ptr(la), B, NDATA, N.ptr(ka), N.ptr(wa), wa.numel(), st))
    ga, gsa = _grads(samp, dev)
    dl = torch.empty(B, K, device=dev)
    dha = torch.empty(B, E, device=dev)
    _ck(L.abcd_sampler_sample_backward(cfg, par, B, gmode, tau, N.ptr(d_feats), N.ptr(dl),
                                           N.ptr(ga["codebook"]), N.ptr(wa), wa.numel(), st))
    _ck(L.abcd_sampler_kl_backward(cfg, par, B, NDATA, N.ptr(d_kl), 1, N.ptr(dl),
                                       N.ptr(ga["posterior_shape_logits"]), N.ptr(wa), wa.numel(), st))
    _ck(L.abcd_sampler_forward_backward(cfg, par, N.ptr(h), B, N.ptr(dl), N.ptr(dha), gsa, 1, N.ptr(wa),
                                            wa.numel(), st))

    # fused: two launches forward, samp_head_bwd + d_h GEMM backward
    wb = N.workspace(nbytes, dev)
    L.abcd_dispatch_reset()
    lb, fb, kb = torch.empty(B, K, device=dev), torch.empty(B, D, device=dev), torch.empty(1, device=dev)
    pb = torch.zeros(3, device=dev)
    _ck(L.abcd_sampler_forward_fused(cfg, par, N.ptr(h), B, gmode, tau, N.ptr(noise), seed, off, NDATA,
                                         N.ptr(lb), N.ptr(fb), N.ptr(kb), N.ptr(pb), N.ptr(wb), wb.numel(), st))
    gb, gsb = _grads(samp, dev)
    dhb = torch.empty(B, E, device=dev)
    _ck(L.abcd_sampler_backward_split(cfg, par, N.ptr(h), B, gmode, tau, NDATA, N.ptr(d_feats), N.ptr(d_kl),
                                          N.ptr(dhb), gsb, N.ptr(wb), wb.numel(), st, None))
    torch.cuda.synchronize()
    ran = N.dispatch()
    assert "samp_head_fwd grid %d" % ((B + 15) // 16) in ran["samp_fwd"][0], ran
    assert ran["samp_bwd"][0].startswith("samp_head_bwd"), ran

    assert _rel(lb, la) < 1e-5
    assert _rel(fb, fa) < 1e-5
    assert abs(float(kb) - float(ka)) <= 1e-5 * abs(float(ka)) + 1e-6, (float(kb), float(ka))
    assert torch.equal(lb.argmax(-1), la.argmax(-1))
    pa = torch.zeros(3, device=dev)  # the per-method perplexity kernel on the same logits
    _ck(L.abcd_perplexities(N.ptr(la), B, K, N.ptr(samp.posterior_shape_logits), N.ptr(pa), st))
    _ck(L.abcd_shape_perplexity(N.ptr(samp.posterior_shape_logits), K, N.ptr(pb[2:]), st))
    assert _rel(pb, pa) < 1e-5, (pb, pa)
    assert _rel(dhb, dha) < 1e-4
    for k in ga:
        assert _rel(gb[k], ga[k]) < 1e-4, (k, _rel(gb[k], ga[k]))


def test_fused_head_repeatable():
    """The KL scalar and the column sums are reduced in tile order by the last
    workgroup: two runs give bit-identical results."""
    from modules import model as M, _native as N
    L = N.lib()
    dev = torch.device("cuda")
    torch.manual_seed(3)
    B, E, Hm, K, D = 512, 1024, 256, 128, 256
    samp = M.ABCDSampler(E, Hm, K, D).to(dev)
    cfg, par = samp._scfg(), samp._sparams()
    h = torch.randn(B, E, device=dev)
    d_feats = torch.randn(B, D, device=dev)
    d_kl = torch.full((), 1.0 / B, device=dev)
    ws = N.workspace(L.abcd_sampler_workspace_bytes(cfg, B), dev)
    outs = []
    for _ in range(2):
        lg, ft, kl = torch.empty(B, K, device=dev), torch.empty(B, D, device=dev), torch.empty(1, device=dev)
        pp = torch.empty(2, device=dev)
        _ck(L.abcd_sampler_forward_fused(cfg, par, N.ptr(h), B, N.SAMPLE_GUMBEL, 0.5, None, 5, 0, 1e4,
                                             N.ptr(lg), N.ptr(ft), N.ptr(kl), N.ptr(pp), N.ptr(ws), ws.numel(),
                                             N.stream()))
        g, gs = _grads(samp, dev)
        dh = torch.empty(B, E, device=dev)
        _ck(L.abcd_sampler_backward_split(cfg, par, N.ptr(h), B, N.SAMPLE_GUMBEL, 0.5, 1e4, N.ptr(d_feats),
                                              N.ptr(d_kl), N.ptr(dh), gs, N.ptr(ws), ws.numel(), N.stream(), None))
        torch.cuda.synchronize()
        outs.append([lg, ft, kl, pp, dh] + [g[k] for k in sorted(g)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("K", [128, 1024])
@pytest.mark.parametrize("on_side", [False, True])
def test_deferred_parameter_gradients_identical(K, on_side):
    """abcd_sampler_backward_split with ABCD_DEFER_PARAMS, then
    abcd_sampler_backward_params (the engine's order: the codebook / W2 / W1
    gradients after the encoder's backward) gives the same bits as the
    one-call backward: the same batched GEMM launch on the same workspace
    stash, only later in stream order -- on `stream` or on a side stream (the
    engine's form: side tiling, 16-deep LDS slabs, the same sums in the same
    order).  d_h is complete after the first call."""
    from modules import model as M, _native as N
    L = N.lib()
    dev = torch.device("cuda")
    torch.manual_seed(11 + K)
    B, E, Hm, D = 512, 1024, 256, 256
    samp = M.ABCDSampler(E, Hm, K, D).to(dev)
    cfg, par = samp._scfg(), samp._sparams()
    h = torch.randn(B, E, device=dev)
    d_feats = torch.randn(B, D, device=dev) / B
    d_kl = torch.full((), 1.0 / B, device=dev)
    ws = N.workspace(L.abcd_sampler_workspace_bytes(cfg, B), dev)
    st = N.stream()
    side = torch.cuda.Stream() if on_side else None
    outs = []
    for defer in (False, True):
        lg, ft, kl = torch.empty(B, K, device=dev), torch.empty(B, D, device=dev), torch.empty(1, device=dev)
        _ck(L.abcd_sampler_forward_fused(cfg, par, N.ptr(h), B, N.SAMPLE_GUMBEL, 0.5, None, 5, 0, 1e4,
                                         N.ptr(lg), N.ptr(ft), N.ptr(kl), None, N.ptr(ws), ws.numel(), st))
        g, gs = _grads(samp, dev)
        dh = torch.empty(B, E, device=dev)
        _ck(L.abcd_sampler_backward_split(cfg, par, N.ptr(h), B, N.SAMPLE_GUMBEL, 0.5, 1e4, N.ptr(d_feats),
                                          N.ptr(d_kl), N.ptr(dh), gs, N.ptr(ws), ws.numel(), st,
                                          N.DEFER_PARAMS if defer else None))
        if defer:
            torch.cuda.synchronize()
            assert all(float(g[k].abs().max()) == 0.0 for k in ("codebook", "mlp0.w1", "mlp0.w2")), \
                "parameter gradients written before abcd_sampler_backward_params"
            _ck(L.abcd_sampler_backward_params(cfg, par, N.ptr(h), B, gs, N.ptr(ws), ws.numel(), st,
                                               side.cuda_stream if side is not None else None))
        torch.cuda.synchronize()  # joins the side stream too
        outs.append([dh] + [g[k] for k in sorted(g)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
