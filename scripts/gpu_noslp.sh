# GPU box: the library built with -fno-slp-vectorize (no packed f32 VALU beside the MFMAs) against the default build
set -e
OUT=gpurun_out/noslp
mkdir -p $OUT
export TMPDIR=/tmp
PKG=$PWD/seq2seq_abcd-vae_amd
for L in libabcd_hip.so libabcd_noslp.so; do
  echo "== $L" >> $OUT/probe.log
  ABCD_HIP_LIB=$PKG/$L timeout -k 10 200 python -u scripts/wg_probe.py 0 1 0 1 2>&1 | grep -v amdgpu.ids >> $OUT/probe.log
done
cat $OUT/probe.log
bash scripts/ab_libs.sh seq2seq_abcd-vae_amd/libabcd_hip.so seq2seq_abcd-vae_amd/libabcd_noslp.so > $OUT/ab.log 2>&1; cat $OUT/ab.log
