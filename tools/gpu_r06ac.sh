#!/bin/bash
# Round 6: the precise engine with the F waves' next-tile x DMA issued after stage 2 (no lo8 refill
# younger than it), against the previous build
# (libbcfft_exp_prev.so): dftp parity first, then dftp / dftx interleaved.
# usage (through gpurun): bash tools/gpu_r06ac.sh TAG
set -o pipefail
TAG=${1:-r06ac}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_dftp.py tests/test_gpu_0_north_star.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/$TAG/pytest.log | head -20; tail -5 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
bash tools/ab_fp32.sh $TAG "dftp dftx" "" libbcfft_exp_prev.so "" libbcfft_exp_prev.so
