#!/usr/bin/env python3
"""Times the library's GEMM routes at the c2 hot-path shapes (HIP events,
median of 20 launches) -- the frame-parallel input projection / offset head
(abcd_gemm_nt, both operands K-contiguous) and the weight gradients
(abcd_gemm_tn, both K-major, K = packed frames)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "seq2seq_abcd-vae_amd"))
from modules import _native as Nn  # noqa: E402

L = 65583
SHAPES = [("nt", "xproj", L, 2048, 144), ("nt", "offset-head", L, 256, 256),
          ("tn", "dW_hh", 1024, 256, L), ("tn", "dW_ih", 1024, 129, L), ("wg", "wg2", 1024, 129, L)]


def run(kind, M, N, K):
    g = torch.Generator(device="cuda").manual_seed(1)
    ws = Nn.workspace(64 * M * N * 4 + (1 << 22), "cuda")
    if kind == "wg":  # abcd_lstm_wgrad: both directions' [dW_ih | db | dW_hh] (F = N, H = M / 4)
        H, F = M // 4, N
        dG = [torch.randn(K, M, device="cuda", generator=g) for _ in range(2)]
        X = torch.randn(K, F, device="cuda", generator=g)
        Hp = [torch.randn(K, H, device="cuda", generator=g) for _ in range(2)]
        wih = [torch.empty(M, F, device="cuda") for _ in range(2)]
        bih = [torch.empty(M, device="cuda") for _ in range(2)]
        whh = [torch.empty(M, H, device="cuda") for _ in range(2)]
        wsb = Nn.workspace(Nn.lib().abcd_lstm_wgrad_workspace_bytes(2, F, H, K), "cuda")
        arr = lambda ts: (ctypes.c_void_p * 2)(*[t.data_ptr() for t in ts])
        keep = [arr(dG), arr(Hp), arr(wih), arr(bih), arr(whh)]
        f = lambda: Nn.lib().abcd_lstm_wgrad(2, F, H, K, keep[0], Nn.ptr(X), F, keep[1], keep[2], keep[3], None,
                                             keep[4], Nn.ptr(wsb), wsb.numel(), Nn.stream())
        C = whh[1]
        ref = lambda: dG[1].double().t() @ Hp[1].double()
        Nn.check(f(), "wgrad")
        torch.cuda.synchronize()
        e1 = ((wih[0].double() - dG[0].double().t() @ X.double()).abs().max() / (dG[0].double().t() @ X.double()).abs().max()).item()
        e2 = ((bih[0].double() - dG[0].double().sum(0)).abs().max() / dG[0].double().sum(0).abs().max()).item()
        print(f"  wg2 rel err: w_ih {e1:.2e}  b {e2:.2e}", flush=True)
    elif kind == "nt":
        A = torch.randn(M, K, device="cuda", generator=g)
        B = torch.randn(N, K, device="cuda", generator=g)
        C = torch.empty(M, N, device="cuda")
        bias = torch.randn(N, device="cuda", generator=g)
        f = lambda: Nn.lib().abcd_gemm_nt(M, N, K, Nn.ptr(A), K, Nn.ptr(B), K, Nn.ptr(C), N, Nn.ptr(bias),
                                          Nn.ptr(ws), ws.numel(), Nn.stream())
        ref = lambda: A.double() @ B.double().t() + bias.double()
    else:
        ldb = (N + 15) // 16 * 16
        A = torch.randn(K, M, device="cuda", generator=g)
        B = torch.randn(K, ldb, device="cuda", generator=g)
        C = torch.empty(M, N, device="cuda")
        f = lambda: Nn.lib().abcd_gemm_tn(M, N, K, Nn.ptr(A), M, Nn.ptr(B), ldb, Nn.ptr(C), N, Nn.ptr(ws),
                                          ws.numel(), Nn.stream())
        ref = lambda: A.double().t() @ B[:, :N].double()
    Nn.check(f(), "gemm")
    torch.cuda.synchronize()
    err = ((C.double() - ref()).abs().max() / ref().abs().max()).item()
    ts = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2], err


if __name__ == "__main__":
    tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("ABCD_")) or "default"
    only = sys.argv[1:]
    for kind, name, M, N, K in SHAPES:
        if only and name not in only:
            continue
        us, err = run(kind, M, N, K)
        print(f"[{tag}] {name:12s} M={M} N={N} K={K}: {us:8.1f} us  (rel err vs f64 {err:.2e})", flush=True)
