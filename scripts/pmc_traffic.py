#!/usr/bin/env python3
"""Per-launch HBM traffic of the persistent recurrent kernels from rocprofv3
PMC passes (run separately, one counter group per pass):

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py ...
    python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/traffic_c2.json c2

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  gfx950 correction
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE tallies 128-B requests at
64 B, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16-B
stores and atomics.  Values are averaged over the dispatches of each kernel.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# role -> the persistent kernels that implement it (bench.py reports by role)
ROLES = {"enc_fwd": ("enc_fwd_persist",), "enc_bwd": ("enc_bwd_persist", "enc_bwd_sk", "enc_bwd_w8"),
         "dec_fwd": ("dec_fwd_persist", "dec_fwd_x6"), "dec_bwd": ("dec_bwd_persist", "dec_bwd_sk", "dec_bwd_fold", "dec_bwd_w16")}
# the step's other large kernels (algorithmic bytes: DESIGN.md s3 "Other kernels")
OTHERS = {"gemm_wg3b": ("gemm_wg3b_kernel",), "gemm_x6r": ("gemm_x6r_kernel",), "gemm_x6r8 (input projection)": ("gemm_x6r8_kernel<5",), "gemm_x6r8 (offset head fwd)": ("gemm_x6r8_kernel<8, 64, 2, 16, 1",), "gemm_x6r8 (offset head bwd)": ("gemm_x6r8_kernel<8, 64, 2, 16, 2",), "gemm_tn": ("gemm_tn_kernel",), "gemm_x6s": ("gemm_x6s_kernel",), "gemm_x6t": ("gemm_x6t_kernel",),
          "gemm_tn_batch": ("gemm_tn_batch_kernel",), "colsum_batch": ("colsum_batch_pass1",),
          "slab_reduce": ("slab_reduce_kernel",)}
KERNELS = tuple(ROLES) + tuple(OTHERS)


def short(name):
    for role, syms in list(ROLES.items()) + list(OTHERS.items()):
        if any("abcd::" + sym in name for sym in syms):
            return role
    return None


def read_pass(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                k = short(row.get("Kernel_Name", ""))
                if k:
                    vals[k].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    fetch_dir, write_dir, out = sys.argv[1:4]
    cfg = sys.argv[4] if len(sys.argv) > 4 else "c2"
    fetch, nf = read_pass(fetch_dir, "FETCH_SIZE")
    write, nw = read_pass(write_dir, "WRITE_SIZE")
    res = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, bench.py --config {cfg}",
           "config": cfg,
           "correction": "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE counts 1/2)",
           "kernels": {}}
    for k in KERNELS:
        if k in fetch and k in write:
            rb, wb = 2 * fetch[k] * 1024, write[k] * 1024
            res["kernels"][k] = {"fetch_size_kib": round(fetch[k], 1), "write_size_kib": round(write[k], 1),
                                 "read_bytes": int(rb), "write_bytes": int(wb),
                                 "hbm_bytes_per_launch": int(rb + wb), "dispatches": min(nf[k], nw[k])}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
