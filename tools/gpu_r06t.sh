#!/bin/bash
# Round 6: precise-engine (dftp) stage-2 schedule variants. Parity of each build on the dftp tests,
# then dftp timing interleaved with the product. usage (through gpurun): bash tools/gpu_r06t.sh TAG LIB...
set -o pipefail
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
for L in "$@"; do
  BCFFT_LIB_PATH=$PWD/llama-fft_amd/lib/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_dftp.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest_$L.log 2>&1 || exit 1
done
bash tools/ab_fp32.sh $TAG "dftp" "" "$@"
