#!/bin/bash
# Round-3 PMC traffic of the kernels added late in the round: b = 256 (4096^2 resident weights,
# 11008 -> 4096 streamed) and b = 64 11008 -> 4096 streamed; FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 runs, kernel trace only beside --pmc.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
run() {   # TAG ALGO K M B IO N
  local tag=$1 algo=$2; shift 2
  local out=gpurun_out/pmc3_$tag
  mkdir -p $out
  local i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    BCFFT_ALGO=$algo timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $out/g$i -o run -- \
        python3 tools/run_fwd.py "$@" 6 > $out/g$i.log 2>&1 || { echo "pmc $tag $grp failed"; return 1; }
  done
}
run b256sq auto 4096 4096 256 bf16 8192 &&
run b256down auto 11008 4096 256 bf16 8192 &&
run b64down auto 11008 4096 64 bf16 8192 &&
run b256up auto 4096 11008 256 bf16 8192 &&
python3 tools/pmc_traffic.py r03b 4096x4096_b256_n8192_bf16=gpurun_out/pmc3_b256sq@dft \
    11008x4096_b256_n8192_bf16=gpurun_out/pmc3_b256down@dft 11008x4096_b64_n8192_bf16=gpurun_out/pmc3_b64down@dft \
    4096x11008_b256_n8192_bf16=gpurun_out/pmc3_b256up@dft > gpurun_out/pmc_traffic_r03b.json
cat gpurun_out/pmc_traffic_r03b.json
