#!/usr/bin/env python3
"""Times abcd_gemm_nt (C = A B^T + bias) at the frame-parallel shapes of the c2
step (input projection 64044 x 2048 x 144, offset head 64044 x 256 x 256) with
HIP events, 20 launches after 3 warm-up ones."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "seq2seq_abcd-vae_amd"))
from modules import _native as Nn  # noqa: E402


def run(M, N, K, reps=20):
    g = torch.Generator(device="cuda").manual_seed(1)
    A = torch.randn(M, K, device="cuda", generator=g)
    B = torch.randn(N, K, device="cuda", generator=g)
    bias = torch.randn(N, device="cuda", generator=g)
    C = torch.empty(M, N, device="cuda")
    ws = Nn.workspace(64 << 20, "cuda")
    call = lambda: Nn.check(Nn.lib().abcd_gemm_nt(M, N, K, Nn.ptr(A), K, Nn.ptr(B), K, Nn.ptr(C), N, Nn.ptr(bias),
                                                  Nn.ptr(ws), ws.numel(), Nn.stream()), "gemm")
    for _ in range(3):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    err = (C[:4096] - (A[:4096].double() @ B.double().t() + bias.double()).float()).abs().max().item()
    return us, err


if __name__ == "__main__":
    tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("ABCD_"))
    for shp in [(64044, 2048, 144), (64044, 256, 256)]:
        us, err = run(*shp)
        print(f"[{tag}] {shp}: {us:8.1f} us  max err {err:.2e}  {2 * shp[0] * shp[1] * shp[2] / us / 1e6:.1f} TF/s")
