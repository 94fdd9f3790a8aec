#!/bin/bash
# One GPU call for the DFT-on-MFMA kernel: parity tests, stamps timeline (fp32, bf16), per-algo
# timing. Each GPU step under its own time limit; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-dm}
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dft.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 120 python3 tools/timeline_dm.py 4096 fp32 8192 > gpurun_out/${TAG}_tl.log 2>&1 &&
timeout -k 10 120 python3 tools/timeline_dm.py 4096 bf16 8192 >> gpurun_out/${TAG}_tl.log 2>&1 &&
timeout -k 10 200 python3 tools/time_algos.py dft stationary > gpurun_out/${TAG}_time.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/${TAG}_tl.log gpurun_out/${TAG}_time.log
exit $rc
