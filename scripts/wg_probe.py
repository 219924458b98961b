#!/usr/bin/env python3
"""Times abcd_lstm_wgrad (the encoder's layer-0 weight gradients, both
directions, gemm_wg2 or gemm_wg3b by ABCD_WG3) at the c2 shape (F = 129,
H = 256, K = 64077 frames) with HIP events: 20 launches after 3 warm-up ones,
for each ABCD_WG3 value given on the command line (default "0 1")."""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "seq2seq_abcd-vae_amd"))
from modules import _native as Nn  # noqa: E402


def main():
    nd, F, H, K = 2, 129, 256, int(os.environ.get("PROBE_K", "64077"))
    M = 4 * H
    g = torch.Generator(device="cuda").manual_seed(3)
    dG = [torch.randn(K, M, device="cuda", generator=g) for _ in range(nd)]
    X = torch.randn(K, F, device="cuda", generator=g)
    Hp = [torch.randn(K, H, device="cuda", generator=g) for _ in range(nd)]
    outs = [[torch.empty(M, F, device="cuda"), torch.empty(M, device="cuda"), torch.empty(M, device="cuda"),
             torch.empty(M, H, device="cuda")] for _ in range(nd)]
    ws = Nn.workspace(Nn.lib().abcd_lstm_wgrad_workspace_bytes(nd, F, H, K), "cuda")
    arr = lambda ts: (ctypes.c_void_p * nd)(*[t.data_ptr() for t in ts])
    keep = [arr(dG), arr(Hp)] + [arr([o[i] for o in outs]) for i in range(4)]
    call = lambda: Nn.check(Nn.lib().abcd_lstm_wgrad(nd, F, H, K, keep[0], Nn.ptr(X), F, keep[1], keep[2], keep[3],
                                                     keep[4], keep[5], Nn.ptr(ws), ws.numel(), Nn.stream()), "wgrad")
    flop = 2.0 * nd * M * (F + 1 + H) * K
    for v in (sys.argv[1:] or ["0", "1"]):
        os.environ["ABCD_WG3"] = v
        for _ in range(3):
            call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(20):
            call()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 20
        ref = dG[0].double().t() @ Hp[0].double()
        err = ((outs[0][3].double() - ref).abs().max() / ref.abs().max()).item()
        print(f"ABCD_WG3={v}: {us:8.1f} us per call (+ reduce)  {flop / us / 1e6:6.1f} TF/s fp32-equiv  "
              f"w_hh rel err {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
