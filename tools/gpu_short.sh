# short launches: config 1 and the 1024-token shard, timed and phase-timelined (stamps build)
set -o pipefail
TAG=${1:-short}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 120 python -u tools/time_config1.py > gpurun_out/$TAG/config1.json 2>&1 &&
TIMELINE_ALGO=dftx timeout -k 10 120 python -u tools/timeline_dm.py 4096 fp32 1024 > gpurun_out/$TAG/timeline_dftx_1024.txt 2>&1 &&
TIMELINE_BUILD=stamps timeout -k 10 120 python -u tools/timeline_stat.py 4096 4096 64 fp32 128 > gpurun_out/$TAG/timeline_stat_cfg1.txt 2>&1
