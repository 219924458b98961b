#!/usr/bin/env python3
"""Diagnostics: per-phase timing of the sampler-head kernels (samp_head_fwd /
samp_head_bwd, 16-row tiles) in the c2 training step: s_memrealtime stamps of
thread 0 of each tile (abcd_debug_persist_prof masks 16 / 32), median and
max over tiles of each phase, and the last tile's tail (the tile-order
reductions it runs).

    python scripts/head_stamps.py
"""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "seq2seq_abcd-vae_amd"))

import bench  # noqa: E402

NAMES = {16: ("samp_head_fwd", ["prologue (slabs + tanh, CT/W2T slices)", "U = Z1 W2^T", "logits = U C",
                                "prior_block (elog)", "rows: softmax / KL / sample", "feats = Y C^T + partials",
                                "last tile: KL / perplexities"]),
         32: ("samp_head_bwd", ["stage d_feats / Z1 / elog", "dY = d_feats C", "rows: dL", "dU = dL C^T",
                                "dZ1 = dU W2 (1 - Z1^2)", "last tile: column sums", "last tile: prior gradient"])}


def main():
    from modules import _native as N, noise
    lib = N.lib()
    lib.abcd_debug_persist_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.abcd_debug_persist_prof.restype = None
    cfg = bench.CONFIGS["c2"]
    dev = torch.device("cuda", 0)
    noise.set_mode("philox")
    noise.manual_seed(1234)
    step = bench.build(cfg, dev)
    b = bench.make_batch(cfg, 0, dev)

    def run():
        step.step(b["data"], b["batch_sizes"], b["is_offset"], b["speakers"], cfg["N"], is_pretraining=False,
                  lr=0.0, momentum=0.0, clip=1.0)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    tiles = 64
    buf = torch.zeros(tiles * 8, dtype=torch.int64, device=dev)
    for mask, (name, phases) in NAMES.items():
        rows = []
        for rep in range(5):
            buf.zero_()
            lib.abcd_debug_persist_prof(ctypes.c_void_p(buf.data_ptr()), mask)
            run()
            torch.cuda.synchronize()
            lib.abcd_debug_persist_prof(None, 0)
            st = buf.view(tiles, 8).cpu().double() * 10.0  # 100 MHz ticks -> ns
            rows.append(st)
        st = torch.stack(rows)  # reps x tiles x 8
        used = st[0, :, 0] > 0
        st = st[:, used]
        t0 = st[:, :, 0].min(dim=1, keepdim=True).values
        print(f"{name}: {int(used.sum())} tiles, {len(rows)} steps; ns from the first tile's start (median over steps)")
        for k, ph in enumerate(phases):
            a, b_ = st[:, :, k], st[:, :, k + 1]
            ok = b_ > 0
            if not ok.any():
                continue
            dur = torch.where(ok, b_ - a, torch.zeros_like(a))
            med = dur[ok].median().item()
            end = torch.where(ok, b_ - t0, torch.zeros_like(b_)).max(dim=1).values.median().item()
            print(f"   {ph:42s} median {med:8.0f}  last tile done at {end:8.0f}")


if __name__ == "__main__":
    main()
