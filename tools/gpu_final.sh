#!/bin/bash
# Round-end evidence in one GPU session: the whole -m gpu suite, smoke(), the bench line, a
# rocprofv3 kernel-stats summary of the headline-only bench and of the full variant sweep.
# usage (through gpurun): bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-final}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --variants 0 --cpu-budget 0 > "$GRAFT_REPO_ROOT/gpurun_out/$TAG/bench_under_rocprof.json" 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/profsweep" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-budget 0 > "$GRAFT_REPO_ROOT/gpurun_out/$TAG/bench_sweep_under_rocprof.json" 2>&1
