#!/usr/bin/env python3
"""CPU baseline calibration: times bench.py's bounded
oracle sample (b = 64 segments of each workload, the ``cpu_baseline`` leg)
on THIS machine's cores, so the bench line can state the box-to-box factor
between the GPU box's host and the survey container the reference's own CPU
numbers (bench.REFERENCE_CPU) were measured in.

    python scripts/cpu_calibrate.py [--threads 8] [c2 c4 c5 ...]
"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "seq2seq_abcd-vae_amd"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("configs", nargs="*", default=["c2", "c4", "c5", "c5gru"])
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    out = {}
    for name in a.configs:
        cfg = bench.CONFIGS[name]
        smp = bench.oracle_sample(cfg)
        _, steps, t = bench.time_oracle(cfg, smp)
        out[name] = {"value": round(steps * smp["b"] / t, 3), "cores": a.threads, "steps": steps,
                     "seconds": round(t, 3), "L": smp["batch"]["L"]}
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
