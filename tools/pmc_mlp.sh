#!/bin/bash
# HBM traffic of the whole BC-MLP at N = 8192: FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 passes (kernel trace only beside --pmc), fused (one launch) and split (gate/up
# + SwiGLU launch, then down launch); tools/pmc_mlp_sum.py sums the kernels of one MLP call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for mode in fused split; do
  out=gpurun_out/pmc_mlp_$mode
  mkdir -p $out
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $out/g$i -o run -- \
        python3 tools/run_mlp.py 8192 $mode 6 > $out/g$i.log 2>&1 || { echo "pmc $mode $grp failed"; exit 1; }
  done
done
python3 tools/pmc_mlp_sum.py gpurun_out/pmc_mlp_fused gpurun_out/pmc_mlp_split > gpurun_out/pmc_mlp_r03.json
cat gpurun_out/pmc_mlp_r03.json
