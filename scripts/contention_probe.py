#!/usr/bin/env python3
"""Per-launch time of the four persistent kernels at c2 widths with EVERY
sequence of length T (so every row group is full for all T steps), for
B = 32 .. 512 (the forward kernels run 64-row groups, 1 .. 8 active at once;
dec_bwd_w16 / enc_bwd_w8 run 32-row groups, 1 .. 16).  If a step's latency were
intrinsic to a group, the launch time would not depend on B; growth with B is
chip-wide contention (the hand-off traffic of the groups sharing the
MALL / HBM)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "seq2seq_abcd-vae_amd"))
import bench  # noqa: E402
from modules import _native as N, noise  # noqa: E402


def main():
    T = int(os.environ.get("PROBE_T", "200"))
    for B in (32, 64, 128, 256, 512):
        cfg = dict(bench.CONFIGS["c2"], B=B, tmin=T, tmax=T)
        step = bench.build(cfg, "cuda")
        batch = bench.make_batch(cfg, 0, "cuda")
        noise.set_mode("philox")
        run = lambda: step.step(batch["data"], batch["batch_sizes"], batch["is_offset"], batch["speakers"], 10000,
                                is_pretraining=False, lr=1e-4, clip=1.0)
        for _ in range(2):
            run()
        torch.cuda.synchronize()
        lib = N.lib()
        lib.abcd_timing_reset()
        lib.abcd_timing_enable(1)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        lib.abcd_timing_enable(0)
        out = []
        for kid, name in ((1, "enc_fwd"), (2, "enc_bwd"), (3, "dec_fwd"), (4, "dec_bwd")):
            res = (N.c_double * 4)()
            lib.abcd_timing_read_kernel(kid, res)
            ms, n = res[0], res[1]
            out.append(f"{name} {ms / max(n, 1) * 1e3:8.1f} us ({ms / max(n, 1) * 1e3 / T:6.2f} us/step)")
        print(f"B={B:4d} fwd groups={max(B // 64, 1)} bwd groups={B // 32}: " + "  ".join(out), flush=True)
        del step


if __name__ == "__main__":
    main()
