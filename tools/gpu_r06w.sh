#!/bin/bash
# Round 6: the precise engine with the last tile's stage 3 split between the F and I waves of a
# slot (DRAIN_SPLIT, as dft / dftx; fp32 bias excluded: it spills there). dftp parity first,
# then dftp / dftx interleaved against the previous build (libbcfft_exp_old.so).
# usage (through gpurun): bash tools/gpu_r06w.sh TAG
set -o pipefail
TAG=${1:-r06w}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_dftp.py tests/test_gpu_0_north_star.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
bash tools/ab_fp32.sh $TAG "dftp dftx" "" libbcfft_exp_old.so "" libbcfft_exp_old.so
