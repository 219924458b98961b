#!/bin/bash
# Build the library of another commit (default HEAD) as seq2seq_abcd-vae_amd/libabcd_b.so for a
# same-box A/B against the working tree's libabcd_hip.so (scripts/gpu_ab_lib.sh).
# usage: bash scripts/build_ab.sh [commit]
set -e
REV=${1:-HEAD}
REPO=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/abcd_ab.XXXX)
mkdir -p $T/pkg
git -C $REPO archive $REV seq2seq_abcd-vae_amd/csrc include | tar -x -C $T
mv $T/seq2seq_abcd-vae_amd/csrc $T/pkg/csrc
make -C $T/pkg/csrc -j8 OUT=$REPO/seq2seq_abcd-vae_amd/libabcd_b.so > $T/build.log 2>&1 || { tail -20 $T/build.log; exit 1; }
rm -rf $T
echo "libabcd_b.so = $REV"
