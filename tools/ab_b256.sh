#!/bin/bash
# A/B of experiment builds on the b = 256 rows in one GPU session.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; shift
for round in 1 2; do
  for L in "$@"; do
    P=$PWD/llama-fft_amd/lib/${L:-libbcfft.so}
    echo "== $L round $round" >> gpurun_out/ab_$TAG.log
    BCFFT_LIB_PATH=$P timeout -k 10 120 python3 tools/time_algos.py dft --b256 >> gpurun_out/ab_$TAG.log 2>&1 || exit 1
  done
done
grep -v amdgpu gpurun_out/ab_$TAG.log
