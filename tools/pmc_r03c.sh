#!/bin/bash
# Round-3 PMC for the b = 64 sweep rows without counters so far: HBM traffic of 4096^2 (dm64) and
# 4096 -> 11008 (dm64g), and utilisation counters of the slowest row, 11008 -> 4096 (dm64k).
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
run b64sq auto 4096 4096 64 bf16 8192 &&
run b64up auto 4096 11008 64 bf16 8192 &&
python3 tools/pmc_traffic.py r03c 4096x4096_b64_n8192_bf16=gpurun_out/pmc3_b64sq@dft \
    4096x11008_b64_n8192_bf16=gpurun_out/pmc3_b64up@dft > gpurun_out/pmc_traffic_r03c.json &&
cat gpurun_out/pmc_traffic_r03c.json || exit 1
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
G2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
G3="TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum"
RUN="11008 4096 64 bf16 8192" bash tools/pmc_groups.sh r3dm64k "$G1" "$G2" "$G3" 2>&1 | grep dm64k
exit 0
