#!/bin/bash
# round-4 utilisation counters of the product kernels (one rocprofv3 --pmc pass per group, each
# under its own kill timeout): the fp32 headline (dftx), the bf16 north star (dm8), config 2
# (dmg), the b = 128 and b = 64 down projections (dmk, dm64k); profiles/r04_pmc_util_<tag>.txt
cd "$GRAFT_REPO_ROOT"
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
G2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
G3="SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_COEXEC_CYCLES"
G4="TCC_HIT_sum TCC_MISS_sum"
mkdir -p gpurun_out/util4
for spec in "dftx:4096 4096 128 fp32 8192" "dm8:4096 4096 128 bf16 8192" "dmg:4096 11008 128 bf16 8192" \
            "dmk:11008 4096 128 bf16 8192" "dm64k:11008 4096 64 bf16 8192"; do
  tag=${spec%%:*}
  RUN="${spec#*:}" bash tools/pmc_groups.sh r4$tag "$G1" "$G2" "$G3" "$G4" 2>&1 | grep "bcfft::bc_forward" > gpurun_out/util4/$tag.txt
  cat gpurun_out/pmc_r4$tag/failures.txt 2>/dev/null && exit 1
done
exit 0
