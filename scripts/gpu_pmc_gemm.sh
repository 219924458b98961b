set -e
O=gpurun_out/pmcg
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 scripts/gemm_bench.py > $O/p1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o run -- python3 scripts/gemm_bench.py > $O/p3.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p4 -o run -- python3 scripts/gemm_bench.py > $O/p4.log 2>&1
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
timeout -s KILL 60 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 scripts/gemm_bench.py > $O/p2.log 2>&1
echo done
