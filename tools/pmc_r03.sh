#!/bin/bash
# Round-3 PMC traffic passes (FETCH_SIZE and WRITE_SIZE in separate rocprofv3 runs, kernel trace
# only beside --pmc): the headline (dftx), the bf16 north star, config 2 (dmg), the down
# projection (dmk) at two tile sizes.
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
run fp32dftx dftx 4096 4096 128 fp32 8192 &&
run fp32dft dft 4096 4096 128 fp32 8192 &&
run bf16 auto 4096 4096 128 bf16 8192 &&
run up auto 4096 11008 128 bf16 8192 &&
run down auto 11008 4096 128 bf16 8192 &&
run down5000 auto 11008 4096 128 bf16 5000 &&
python3 tools/pmc_traffic.py r03 4096x4096_b128_n8192_fp32=gpurun_out/pmc3_fp32dftx@dftx \
    4096x4096_b128_n8192_fp32_dft=gpurun_out/pmc3_fp32dft@dft 4096x4096_b128_n8192_bf16=gpurun_out/pmc3_bf16@dft \
    4096x11008_b128_n8192_bf16=gpurun_out/pmc3_up@dft 11008x4096_b128_n8192_bf16=gpurun_out/pmc3_down@dft \
    11008x4096_b128_n5000_bf16=gpurun_out/pmc3_down5000@dft > gpurun_out/pmc_traffic_r03.json
