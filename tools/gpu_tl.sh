# phase timelines of the fp32 DFT kernel (stamps build) at the headline and its 1024-token shard
set -o pipefail
TAG=${1:-tl}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
for n in 8192 1024; do
  TIMELINE_ALGO=dftx timeout -k 10 120 python -u tools/timeline_dm.py 4096 fp32 $n > gpurun_out/$TAG/timeline_dftx_$n.txt 2>&1 || exit 1
done
