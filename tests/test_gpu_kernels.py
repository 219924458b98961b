"""Kernel-level checks of the fp32 MFMA GEMM core and the Philox noise against
plain torch fp32 (GEMM shapes of the hot path, ragged edges)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K", [(16, 16, 16), (33, 70, 48), (512, 1024, 256), (65, 2048, 144), (7, 5, 3),
                                   (1000, 129, 385), (300, 512, 1024), (8001, 520, 144), (7000, 256, 256),
                                   (9000, 300, 136), (64044, 2048, 144), (22854, 1536, 144), (30001, 384, 256)])
def test_gemm_nt_vs_torch(M, N, K):
    """C = A B^T + bias; the shapes from (8001, 520, 144) on take the
    frame-parallel route (>= 240 128-wide tiles): K <= 256 the frame-streaming
    split-fp32 gemm_x6r8 (ragged M / N, a partial last K chunk -- K in (128,
    144] on 16-deep MFMAs --, the c2 input projection, the GRU encoder's 3 x 2 x 256 = 1536 gate columns: slice
    counts that do not divide the grid evenly), else the fragment-staged
    gemm_x6f."""
    from modules import _native as Nn
    g = torch.Generator(device="cuda").manual_seed(M * 1000 + N + K)
    A = torch.randn(M, K, device="cuda", generator=g)
    B = torch.randn(N, K, device="cuda", generator=g)
    bias = torch.randn(N, device="cuda", generator=g)
    C = torch.empty(M, N, device="cuda")
    ws = Nn.workspace(64 << 20, "cuda")
    Nn.check(Nn.lib().abcd_gemm_nt(M, N, K, Nn.ptr(A), K, Nn.ptr(B), K, Nn.ptr(C), N, Nn.ptr(bias), Nn.ptr(ws),
                                   ws.numel(), Nn.stream()), "gemm")
    ref = (A.double() @ B.double().t() + bias.double()).float()
    err = (C - ref).abs().max().item()
    assert err <= 1e-5 * K ** 0.5 * 4 + 1e-5, err


@pytest.mark.parametrize("wg", ["3", "2"])
@pytest.mark.parametrize("nd,F,H,K", [(2, 129, 256, 65583), (1, 129, 256, 3001), (2, 130, 256, 777), (2, 33, 48, 500),
                                       (1, 20, 24, 64), (2, 129, 256, 31), (1, 143, 256, 100003)])
def test_lstm_wgrad_vs_torch(nd, F, H, K, wg, monkeypatch):
    """abcd_lstm_wgrad (the LSTM layer's w_ih, b_ih, b_hh, w_hh gradients from
    the gate gradients, model.py:53,60-66): gemm_wg3b (default) or gemm_wg2
    (ABCD_WG3=0) at F <= 143, H = 256 (the c2 shape first, both directions;
    a K below one chunk; the widest F with a K range that is not a multiple
    of 32), the split-GEMM route elsewhere -- against float64 torch."""
    # "3": the default (gemm_wg3b, 256-row tiles)
    monkeypatch.setenv("ABCD_WG3", "0" if wg == "2" else "1")
    wg = {"3": "3b", "2": "2"}[wg]
    import ctypes
    from modules import _native as Nn
    g = torch.Generator(device="cuda").manual_seed(nd * 7 + F + H + K)
    M = 4 * H
    dG = [torch.randn(K, M, device="cuda", generator=g) for _ in range(nd)]
    X = torch.randn(K, F, device="cuda", generator=g)
    Hp = [torch.randn(K, H, device="cuda", generator=g) for _ in range(nd)]
    wih = [torch.full((M, F), float("nan"), device="cuda") for _ in range(nd)]
    bih = [torch.full((M,), float("nan"), device="cuda") for _ in range(nd)]
    bhh = [torch.full((M,), float("nan"), device="cuda") for _ in range(nd)]
    whh = [torch.full((M, H), float("nan"), device="cuda") for _ in range(nd)]
    ws = Nn.workspace(Nn.lib().abcd_lstm_wgrad_workspace_bytes(nd, F, H, K), "cuda")
    arr = lambda ts: (ctypes.c_void_p * nd)(*[t.data_ptr() for t in ts])
    keep = [arr(dG), arr(Hp), arr(wih), arr(bih), arr(bhh), arr(whh)]
    Nn.lib().abcd_dispatch_reset()
    Nn.check(Nn.lib().abcd_lstm_wgrad(nd, F, H, K, keep[0], Nn.ptr(X), F, keep[1], keep[2], keep[3], keep[4], keep[5],
                                      Nn.ptr(ws), ws.numel(), Nn.stream()), "lstm wgrad")
    torch.cuda.synchronize()
    route = Nn.dispatch()["enc_wgrad"][0]
    assert route == (f"gemm_wg{wg}<144,{H}> x{nd}" if (H == 256 and F <= 143 and (F + 16) // 16 * 16 == 144)
                     else "gemm split (x6s/x6t)"), route
    rel = lambda a, b: ((a.double() - b).abs().max() / b.abs().max()).item()
    for d in range(nd):
        gd = dG[d].double()
        assert rel(wih[d], gd.t() @ X.double()) < 1e-5
        assert rel(whh[d], gd.t() @ Hp[d].double()) < 1e-5
        assert rel(bih[d], gd.sum(0)) < 1e-5
        assert torch.equal(bih[d], bhh[d])


@pytest.mark.parametrize("M,N,K,lda,ldb", [(1024, 256, 64045, 1024, 256), (1024, 129, 20000, 1024, 144),
                                           (129, 256, 7001, 144, 512), (33, 48, 45, 48, 48), (256, 256, 513, 260, 256),
                                           (1024, 1024, 4096, 1024, 1024)])
def test_gemm_tn_vs_torch(M, N, K, lda, ldb):
    """weight-gradient GEMM C = A^T B over K rows (LDS-staged K-major kernel for K >= 512)"""
    from modules import _native as Nn
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randn(K, lda, device="cuda", generator=g)
    B = torch.randn(K, ldb, device="cuda", generator=g)
    C = torch.empty(M, N, device="cuda")
    ws = Nn.workspace(64 * M * N * 4 + (1 << 20), "cuda")
    Nn.check(Nn.lib().abcd_gemm_tn(M, N, K, Nn.ptr(A), lda, Nn.ptr(B), ldb, Nn.ptr(C), N, Nn.ptr(ws), ws.numel(),
                                   Nn.stream()), "gemm_tn")
    ref = (A[:, :M].double().t() @ B[:, :N].double()).float()
    err = (C - ref).abs().max().item()
    assert err <= 2e-6 * K ** 0.5 * 4 + 1e-5, err


def test_linear_tanh():
    from modules import _native as Nn
    x = torch.randn(100, 256, device="cuda")
    W = torch.randn(64, 256, device="cuda") * 0.05
    b = torch.randn(64, device="cuda")
    y = torch.empty(100, 64, device="cuda")
    ws = Nn.workspace(16 << 20, "cuda")
    Nn.check(Nn.lib().abcd_linear(100, 64, 256, Nn.ptr(x), 256, Nn.ptr(W), 256, Nn.ptr(b), 1, Nn.ptr(y), 64,
                                  Nn.ptr(ws), ws.numel(), Nn.stream()), "linear")
    assert (y - torch.tanh(x @ W.t() + b)).abs().max().item() < 1e-5


def test_philox_normal_moments():
    from modules import _native as Nn
    n = 1 << 22
    x = torch.empty(n, device="cuda")
    Nn.check(Nn.lib().abcd_fill_normal(Nn.ptr(x), n, 1234, 0, Nn.stream()), "normal")
    assert abs(x.mean().item()) < 5e-3
    assert abs(x.std().item() - 1) < 5e-3
    y = torch.empty(n, device="cuda")
    Nn.check(Nn.lib().abcd_fill_normal(Nn.ptr(y), n, 1234, 0, Nn.stream()), "normal")
    assert torch.equal(x, y)  # counter-based: reproducible


@pytest.mark.parametrize("B,K", [(512, 128), (100, 16), (37, 1024), (5, 200)])
def test_perplexities_vs_torch_f64(B, K):
    """abcd_perplexities (learning.py:171-178): exp of the mean per-row entropy
    of softmax(logits), of the entropy of the batch-mean probabilities, and of
    the entropy of softmax(posterior_shape_logits); float64 torch reference."""
    from modules import _native as Nn
    g = torch.Generator(device="cuda").manual_seed(3)
    logits = torch.randn(B, K, device="cuda", generator=g) * 3
    psl = torch.randn(K, device="cuda", generator=g)
    out = torch.zeros(3, device="cuda")
    Nn.check(Nn.lib().abcd_perplexities(Nn.ptr(logits), B, K, Nn.ptr(psl), Nn.ptr(out), Nn.stream()), "perplex")
    torch.cuda.synchronize()
    q = torch.softmax(logits.double(), -1)
    ent = -(q * torch.log_softmax(logits.double(), -1)).sum(-1).mean()
    bm = q.mean(0)
    pp = torch.softmax(psl.double(), -1)
    ref = torch.stack([ent.exp(), (-(bm * bm.log()).sum()).exp(), (-(pp * pp.log()).sum()).exp()])
    assert torch.allclose(out.double().cpu(), ref.cpu(), rtol=1e-5, atol=0), (out, ref)
