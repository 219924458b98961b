#!/usr/bin/env python3
"""Diagnostics: per-phase timing of the persistent recurrent kernels.

Runs the bench.py c2 workload, enables the s_memtime stamps of one persistent
kernel at a time (abcd_debug_persist_prof), and prints, per kernel, the median
over workgroups of each phase's cycles averaged over the time steps, plus
the kernel's event-timed duration (to convert cycles to microseconds).

    python scripts/persist_stamps.py [config]      (default c2; e.g. c5)
"""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "seq2seq_abcd-vae_amd"))

import bench  # noqa: E402

NAMES = {1: ("enc_fwd", ["gxload+wait", "mma", "cell+st", "publish+stash"]),
         2: ("enc_bwd", ["epiload+wait+partials", "cell-bwd", "partial-mma+st", "publish"]),
         4: ("dec_fwd", ["cell", "mlp-wait", "mlp", "emit-wait", "emit"]),
         8: ("dec_bwd", ["P0", "P1-wait", "P1", "P2-wait", "P2"])}


def main():
    from modules import _native as N, noise
    lib = N.lib()
    lib.abcd_debug_persist_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.abcd_debug_persist_prof.restype = None
    cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
    dev = torch.device("cuda", 0)
    noise.set_mode("philox")
    noise.manual_seed(1234)
    step = bench.build(cfg, dev)
    b = bench.make_batch(cfg, 0, dev)
    T = b["T"]

    def run():
        step.step(b["data"], b["batch_sizes"], b["is_offset"], b["speakers"], cfg["N"], is_pretraining=False,
                  lr=0.0, momentum=0.0, clip=1.0)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    # which XCD each block of a 256-block grid lands on is not observable here
    grid = 256
    buf = torch.zeros(grid * T * 8, dtype=torch.int64, device=dev)
    for mask, (name, phases) in NAMES.items():
        buf.zero_()
        lib.abcd_debug_persist_prof(ctypes.c_void_p(buf.data_ptr()), mask)
        run()
        torch.cuda.synchronize()
        lib.abcd_debug_persist_prof(None, 0)
        st = buf.view(grid, T, 8).cpu().double() * 10.0  # s_memrealtime ticks (100 MHz) -> ns
        nst = len(phases) + 1
        s = st[:, :, :nst]
        ok = (s > 0).all(dim=2)
        d = s[:, :, 1:] - s[:, :, :-1]  # phase k = stamp k+1 - stamp k
        # step wall: stamp0 of step i+1 - stamp0 of step i
        wall = s[:, 1:, 0] - s[:, :-1, 0]
        okw = ok[:, 1:] & ok[:, :-1]
        res = []
        for k in range(nst - 1):
            v = d[:, :, k][ok]
            res.append(float(v.median()) if v.numel() else float("nan"))
        w = wall[okw]
        # steps split into early (full batch) / late halves
        print(f"{name}: valid (wg,step) {int(ok.sum())}/{grid * T}; median ns per phase:")
        print("   " + "  ".join(f"{p}={c:.0f}" for p, c in zip(phases, res)))
        first = s[:, 0, 0][ok[:, 0]].min()
        last = s[:, -1, nst - 1][ok[:, -1]].max()
        print(f"   span first->last stamp {float(last - first):.0f} ns")
        # start skew: when each workgroup stamped its first step (a late one was
        # placed late, e.g. behind side-stream work holding its CU)
        s00 = s[:, 0, 0][ok[:, 0]] - first
        q = torch.quantile(s00, torch.tensor([0.5, 0.9, 1.0], dtype=s00.dtype))
        print(f"   start skew over workgroups: median {float(q[0]):.0f}  p90 {float(q[1]):.0f}  max {float(q[2]):.0f} ns")
        if w.numel():
            print(f"   step wall median {float(w.median()):.0f} ns, mean {float(w.mean()):.0f} ns")
        # first 40 steps (full batch)
        early = [float(d[:, :40, k][ok[:, :40]].median()) for k in range(nst - 1)]
        print("   first-40-steps: " + "  ".join(f"{p}={c:.0f}" for p, c in zip(phases, early)))
        if name in ("dec_fwd", "dec_bwd"):
            sel = slice(0, 40) if name == "dec_fwd" else slice(T - 40, T)
            full = st[:, sel, :]
            okf = (full[:, :, :8] > 0).all(dim=2)
            def med(a, b):
                v = (full[:, :, a] - full[:, :, b])[okf]
                return float(v.median()) if v.numel() else float("nan")
            # critical path: per (group, step) the LAST member to reach each
            # stamp (groups = blockIdx % 8 under the fallback roles)
            w16 = name == "dec_bwd" and "w16" in N.dispatch().get("dec_bwd", ("",))[0]
            if w16:  # dec_bwd_w16: 16 groups of 16 members (block b: member (b >> 3) % 16, group b % 8 + 8 (b >> 7))
                g8 = st[:, :, :6].reshape(2, 16, 8, T, 6).permute(1, 0, 2, 3, 4).reshape(16, 16, T, 6)
            else:
                g8 = st[:, :, :6].reshape(32, 8, T, 6)  # [member][group][step][stamp]
            okg = (g8 > 0).all(dim=3).all(dim=0)
            last = g8.max(dim=0).values  # [group][step][stamp]
            first = g8.min(dim=0).values
            def cp(a, b, src=last):
                v = (src[:, :, a] - src[:, :, b])[okg]
                return float(v.median()) if v.numel() else float("nan")
            nxt = last[:, 1:, 0] - last[:, :-1, 5]
            okn = okg[:, 1:] & okg[:, :-1]
            print(f"   critical path (last member): 0->1 {cp(1, 0):.0f}  1->2 {cp(2, 1):.0f}  2->3 {cp(3, 2):.0f}  "
                  f"3->4 {cp(4, 3):.0f}  4->5 {cp(5, 4):.0f}  5->next0 {float(nxt[okn].median()):.0f}")
            for k in (1, 3, 5):
                am = g8[:, :, :, k].argmax(dim=0)[okg]
                h = torch.bincount(am, minlength=g8.shape[0])
                top = torch.argsort(h, descending=True)[:6]
                print(f"   last member at stamp {k}: " + " ".join(f"m{int(m)}:{int(h[m])}" for m in top))
            sp = [(last[:, :, k] - first[:, :, k])[okg] for k in range(6)]
            print("   member spread at each stamp (last-first): " + "  ".join(f"{k}:{float(v.median()):.0f}" for k, v in enumerate(sp)))
            if name == "dec_fwd":
                print(f"   full-batch: cell-mma={med(7, 0):.0f} cell-epi+pub={med(1, 7):.0f} "
                      f"mlp-mma={med(6, 2):.0f} mlp-epi+pub={med(3, 6):.0f} step={med(5, 0):.0f}")
            else:
                if os.environ.get("ABCD_STAMP_DIAG"):  # a library built with -DABCD_STAMP_DIAG (dec_bwd_w16)
                    print(f"   full-batch P1: dZ-mma={med(6, 2):.0f} barrier+fold+stores={med(7, 6):.0f} "
                          f"publish={med(3, 7):.0f}")
                else:
                    print(f"   full-batch: P0pub-to-HX-done={med(6, 1):.0f} P1-wait-after-HX={med(2, 6):.0f} "
                          f"P2-dh-sum={med(7, 4):.0f} P2-cell+dx-partials+pub={med(5, 7):.0f}")
    # event timing of the persistent kernels
    lib.abcd_timing_reset()
    lib.abcd_timing_enable(1)
    run()
    torch.cuda.synchronize()
    lib.abcd_timing_enable(0)
    res = (ctypes.c_double * 4)()
    lib.abcd_timing_read(res)
    print(f"timed launches {int(res[1])}: total {res[0]:.3f} ms")


if __name__ == "__main__":
    main()
