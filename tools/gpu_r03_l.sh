#!/bin/bash
# round 3: the down projection's K-chunk split at short grids (tests + timing), MLP / module tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_dmk.py tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03l_pytest.log 2>&1 || { tail -40 gpurun_out/r03l_pytest.log; exit 1; }
tail -2 gpurun_out/r03l_pytest.log
timeout -k 10 200 python -u tools/time_dmk_split.py > gpurun_out/r03l_dmk_split.log 2>&1 || { cat gpurun_out/r03l_dmk_split.log; exit 1; }
grep N gpurun_out/r03l_dmk_split.log
