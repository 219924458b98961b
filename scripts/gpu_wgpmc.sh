# GPU box: gemm_wg2 vs gemm_wg3 alone at the c2 shape, then PMC passes of each
set -e
OUT=gpurun_out/wgpmc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/wg_probe.py 0 1 0 1 > $OUT/probe.log 2>&1; cat $OUT/probe.log
for v in 0 1; do
  ABCD_WG3=$v timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc$v -o run -- python3 scripts/wg_probe.py $v > $OUT/pmc$v.log 2>&1
  ABCD_WG3=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmcb$v -o run -- python3 scripts/wg_probe.py $v > $OUT/pmcb$v.log 2>&1
done
python3 - <<'PY'
import csv, glob, collections
for v in "01":
    acc = collections.defaultdict(list)
    for d in (f"gpurun_out/wgpmc/pmc{v}", f"gpurun_out/wgpmc/pmcb{v}"):
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                if "gemm_wg" in row["Kernel_Name"]:
                    acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    m = {k: sum(x) / len(x) for k, x in acc.items()}
    wall = m.get("GRBM_GUI_ACTIVE", 1) / 8
    print(f"ABCD_WG3={v}", {k: f"{x:.4g}" for k, x in sorted(m.items())})
    print(f"   mfma_busy {m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (1024 * wall):.3f}  wall_cycles {wall:.4g}")
PY
echo wgpmc done
