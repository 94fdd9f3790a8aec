#!/bin/bash
# utilisation counters of the bf16 DFT kernels: dm8 (4096^2) and dmg (4096->11008), b = 128
cd "$GRAFT_REPO_ROOT"
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
G2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
G3="SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_COEXEC_CYCLES"
RUN="4096 4096 128 bf16 8192" bash tools/pmc_groups.sh r3dm8 "$G1" "$G2" "$G3" > gpurun_out/pmc_r3_dm8.txt 2>&1
RUN="4096 11008 128 bf16 8192" bash tools/pmc_groups.sh r3dmg "$G1" "$G2" "$G3" > gpurun_out/pmc_r3_dmg.txt 2>&1
RUN="4096 4096 128 fp32 8192" bash tools/pmc_groups.sh r3dftx "$G1" "$G2" "$G3" > gpurun_out/pmc_r3_dftx.txt 2>&1
cat gpurun_out/pmc_r3_dm8.txt gpurun_out/pmc_r3_dmg.txt gpurun_out/pmc_r3_dftx.txt | grep -v "^$"
cat gpurun_out/pmc_r3*/failures.txt 2>/dev/null
exit 0
