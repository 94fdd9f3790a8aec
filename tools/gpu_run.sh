#!/bin/bash
# One GPU session: the given pytest selection first (default: every -m gpu test), then smoke(),
# the bench line and a rocprofv3 kernel-trace summary of bench.py, all under gpurun_out/$TAG.
# Usage (through gpurun): bash tools/gpu_run.sh TAG [pytest args...]
set -o pipefail
TAG=${1:-run}; shift
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
SEL=${*:-tests}
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -v --timeout 150 --timeout-method thread -s > gpurun_out/$TAG/pytest_gpu.log 2>&1 &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --variants 0 --cpu-budget 0 > "$GRAFT_REPO_ROOT/gpurun_out/$TAG/bench_under_rocprof.json" 2>&1
