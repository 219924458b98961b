#!/usr/bin/env python3
"""MFMA utilisation of the c2 step's kernels from ONE rocprofv3 PMC pass:

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU \\
        SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_mfma -o run -- python3 bench.py ...
    python scripts/pmc_mfma.py gpurun_out/pmc_mfma profiles/pmc_mfma_c2.json c2

Per kernel (mean per dispatch):
  wall_cycles = GRBM_GUI_ACTIVE / 8  (rocprofv3 sums the counter over the 8 XCDs;
                MI355X_MICROARCH.md "DVFS give-back")
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x wall_cycles): the
                fraction of the chip's matrix-core cycles the kernel kept busy
                (SQ_VALU_MFMA_BUSY_CYCLES counts each MFMA's pipe cycles, summed
                over SIMDs: 16 per v_mfma_f32_16x16x32_bf16, 32 per
                v_mfma_f32_16x16x4_f32 -- cycles_per_mfma below checks it)
  valu_per_mfma = (SQ_INSTS_VALU - SQ_INSTS_MFMA) / SQ_INSTS_MFMA
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

COUNTERS = ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_INSTS_MFMA", "SQ_INSTS_VALU",
            "SQ_WAVE_CYCLES")
SIMDS = 1024
# kernel-name fragment -> the name reported (bench.py's roles for the persistent kernels)
NAMES = (("abcd::enc_fwd_persist", "enc_fwd"), ("abcd::enc_bwd_sk", "enc_bwd"), ("abcd::enc_bwd_w8", "enc_bwd"), ("abcd::enc_bwd_persist", "enc_bwd"),
         ("abcd::dec_fwd_x6", "dec_fwd"), ("abcd::dec_fwd_persist", "dec_fwd"), ("abcd::dec_bwd_fold", "dec_bwd"),
         ("abcd::dec_bwd_sk", "dec_bwd"), ("abcd::dec_bwd_persist", "dec_bwd"), ("abcd::dec_bwd_w16", "dec_bwd"), ("gemm_wg2_kernel", "gemm_wg2"), ("gemm_wg3b_kernel", "gemm_wg3b"),
         ("gemm_x6r_kernel", "gemm_x6r"), ("gemm_x6r8_kernel<5", "gemm_x6r8 (input projection)"), ("gemm_x6r8_kernel<8, 64, 2, 16, 1", "gemm_x6r8 (offset head fwd)"), ("gemm_x6r8_kernel<8, 64, 2, 16, 2", "gemm_x6r8 (offset head bwd)"), ("samp_head_fwd", "samp_head_fwd"), ("samp_head_bwd", "samp_head_bwd"),
         ("gemm_tn_kernel", "gemm_tn"), ("gemm_x6s_kernel", "gemm_x6s"), ("gemm_x6t_kernel", "gemm_x6t"),
         ("gemm_tn_batch_kernel", "gemm_tn_batch"), ("colsum_batch_pass1", "colsum_batch"),
         ("slab_reduce_kernel", "slab_reduce"))


def short(name):
    for frag, n in NAMES:
        if frag in name:
            return n
    return None


def main():
    d, out = sys.argv[1:3]
    cfg = sys.argv[3] if len(sys.argv) > 3 else "c2"
    vals = defaultdict(lambda: defaultdict(list))
    symbol = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", ""))
                if k is None or row.get("Counter_Name") not in COUNTERS:
                    continue
                vals[k][(row["Counter_Name"], row.get("Dispatch_Id"))].append(float(row["Counter_Value"]))
                symbol.setdefault(k, row["Kernel_Name"][:120])
    res = {"source": f"rocprofv3 --pmc {' '.join(COUNTERS)} (one pass), bench.py --config {cfg}",
           "config": cfg,
           "formula": "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)",
           "kernels": {}}
    for k, per in vals.items():
        tot = defaultdict(list)
        for (c, _), v in per.items():
            tot[c].append(sum(v))  # a dispatch's counter summed over its rows (dimensions)
        m = {c: sum(v) / len(v) for c, v in tot.items()}
        if not all(c in m for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE")):
            continue
        wall = m["GRBM_GUI_ACTIVE"] / 8
        e = {"symbol": symbol[k], "dispatches": len(tot["GRBM_GUI_ACTIVE"]), "wall_cycles": round(wall),
             "mfma_busy_cycles": round(m["SQ_VALU_MFMA_BUSY_CYCLES"]),
             "mfma_busy": round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * wall), 4)}
        if m.get("SQ_INSTS_MFMA"):
            e["mfma_insts"] = round(m["SQ_INSTS_MFMA"])
            e["cycles_per_mfma"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / m["SQ_INSTS_MFMA"], 2)
            if "SQ_INSTS_VALU" in m:
                e["valu_per_mfma"] = round((m["SQ_INSTS_VALU"] - m["SQ_INSTS_MFMA"]) / m["SQ_INSTS_MFMA"], 2)
        res["kernels"][k] = e
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
