#!/bin/bash
# One GPU-box session: smoke -> parity tests -> bench -> rocprofv3 kernel trace of the bench.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 &&
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1 &&
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o bench -- \
    python3 bench.py --steps 20 --warmup 5 --variants 0 --cpu-budget 0 > gpurun_out/prof_bench_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log 2>/dev/null
cat gpurun_out/bench_$TAG.json 2>/dev/null
exit $rc
