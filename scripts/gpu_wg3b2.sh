# GPU box: gemm_wg3b alone, previous build vs the B split in the MFMA gaps (alternating)
set -e
OUT=gpurun_out/wg3b2
mkdir -p $OUT
PKG=$PWD/seq2seq_abcd-vae_amd
: > $OUT/probe.log
for k in 1 2; do
for L in libabcd_old.so libabcd_hip.so; do
  echo "== $L" >> $OUT/probe.log
  ABCD_HIP_LIB=$PKG/$L timeout -k 10 200 python -u scripts/wg_probe.py 1 1 2>&1 | grep -v amdgpu.ids >> $OUT/probe.log
done
done
cat $OUT/probe.log
