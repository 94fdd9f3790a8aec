#!/bin/bash
# Round 6: the precise engine with the next bin's A rows read one bin ahead (two A buffers, a 3-bin
# lo8 ring) on top of the drain split: dftp parity, then dftp / dftx against the drain-only and
# the previous builds.
# usage (through gpurun): bash tools/gpu_r06x.sh TAG
set -o pipefail
TAG=${1:-r06x}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_dftp.py tests/test_gpu_0_north_star.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
bash tools/ab_fp32.sh $TAG "dftp dftx" "" libbcfft_exp_drain.so libbcfft_exp_old.so
