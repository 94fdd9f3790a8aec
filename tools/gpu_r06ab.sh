#!/bin/bash
# Round 6: does waiting for stage 2's lo8 refills drain the F waves' x DMA (loads return in order,
# and the compiler's counted waits do not see the asm DMA)? Timing-only build "norefill": bins
# 4-7 read the ring slots of bins 0-3 (wrong by construction), no load is issued in stage 2.
# usage (through gpurun): bash tools/gpu_r06ab.sh TAG
set -o pipefail
TAG=${1:-r06ab}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out || exit 1
bash tools/ab_fp32.sh $TAG "dftp dftx" "" libbcfft_exp_norefill.so
