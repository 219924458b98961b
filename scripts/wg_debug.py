#!/usr/bin/env python3
"""gemm_wg3 error map at a small K: max relative error of [dW_ih | db | dW_hh]
per (32-row block, 16-column block) against float64, for the wave forms."""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "seq2seq_abcd-vae_amd"))
from modules import _native as Nn  # noqa: E402


def main():
    nd, F, H = 1, 129, 256
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    M = 4 * H
    g = torch.Generator(device="cuda").manual_seed(3)
    dG = [torch.randn(K, M, device="cuda", generator=g)]
    X = torch.randn(K, F, device="cuda", generator=g)
    Hp = [torch.randn(K, H, device="cuda", generator=g)]
    outs = [[torch.full((M, F), float("nan"), device="cuda"), torch.empty(M, device="cuda"),
             torch.empty(M, device="cuda"), torch.full((M, H), float("nan"), device="cuda")]]
    ws = Nn.workspace(Nn.lib().abcd_lstm_wgrad_workspace_bytes(nd, F, H, K), "cuda")
    arr = lambda ts: (ctypes.c_void_p * nd)(*[t.data_ptr() for t in ts])
    keep = [arr(dG), arr(Hp)] + [arr([o[i] for o in outs]) for i in range(4)]
    Nn.check(Nn.lib().abcd_lstm_wgrad(nd, F, H, K, keep[0], Nn.ptr(X), F, keep[1], keep[2], keep[3], keep[4], keep[5],
                                      Nn.ptr(ws), ws.numel(), Nn.stream()), "wgrad")
    torch.cuda.synchronize()
    got = torch.cat([outs[0][0], outs[0][1][:, None], torch.zeros(M, 144 - F - 1, device="cuda"), outs[0][3]], 1)
    ref = dG[0].double().t() @ torch.cat([X.double(), torch.ones(K, 1, device="cuda", dtype=torch.float64),
                                          torch.zeros(K, 144 - F - 1, device="cuda", dtype=torch.float64),
                                          Hp[0].double()], 1)
    err = (got.double() - ref).abs()
    scale = ref.abs().max().item()
    print(f"K={K} {os.environ.get('ABCD_WG3W', 'default')}: max rel {err.max().item() / scale:.2e}")
    rows = err.view(M // 32, 32, 400).amax(1)  # [32-row block][col]
    for rb in range(0, 8):
        line = "".join("x" if rows[rb, 16 * c:16 * c + 16].max().item() > 1e-4 * scale else "." for c in range(25))
        print(f"rows {32 * rb:4d}: {line}")
    print("bad row blocks:", [rb for rb in range(M // 32) if rows[rb].max().item() > 1e-4 * scale][:40])


if __name__ == "__main__":
    main()
