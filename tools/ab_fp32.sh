#!/bin/bash
# A/B of DFT-kernel builds at the fp32 headline (N = 8192) and its 1024-token shard, interleaved
# rounds, each library with the given engines. usage: tools/ab_fp32.sh TAG "algos" lib1 lib2 ...
# (lib names under llama-fft_amd/lib/, "" = the product build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; ALGOS=$2; shift 2
for round in 1 2; do
  for L in "$@"; do
    echo "== ${L:-product} round $round" >> gpurun_out/ab_$TAG.log
    BCFFT_LIB_PATH=$PWD/llama-fft_amd/lib/${L:-libbcfft.so} timeout -k 10 180 python3 tools/time_algos.py $ALGOS --fp32n >> gpurun_out/ab_$TAG.log 2>&1 || exit 1
  done
done
grep -v amdgpu gpurun_out/ab_$TAG.log
