#!/bin/bash
# Round-5 counter passes: HBM traffic (FETCH_SIZE, WRITE_SIZE), L2 hits and the instruction mix
# of the headline kernel and the bf16 rows the verdict names (dm8, dmg, dm64k).
# usage (GPU box): bash tools/pmc_r05.sh  -> gpurun_out/pmc_r05_<row>/ (tools/pmc_groups.sh)
cd "$GRAFT_REPO_ROOT" || exit 1
G=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
   "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
   "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE")
RUN="4096 4096 128 fp32 8192" bash tools/pmc_groups.sh r05_dftx "${G[@]}" > gpurun_out/pmc_r05_dftx.txt 2>&1 &&
RUN="11008 4096 64 bf16 8192" bash tools/pmc_groups.sh r05_dm64k "${G[@]}" > gpurun_out/pmc_r05_dm64k.txt 2>&1 &&
RUN="4096 4096 128 bf16 8192" bash tools/pmc_groups.sh r05_dm8 "${G[@]}" > gpurun_out/pmc_r05_dm8.txt 2>&1 &&
RUN="4096 11008 128 bf16 8192" bash tools/pmc_groups.sh r05_dmg "${G[@]}" > gpurun_out/pmc_r05_dmg.txt 2>&1
cat gpurun_out/pmc_r05_*.txt
