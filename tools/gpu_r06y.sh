#!/bin/bash
# Round 6: where the precise engine's weight term goes, two timing-only builds of bcfft_dm.hip
# (dftp results wrong by construction or unchecked): "nocvt" takes A's fp8 operand as the fp16
# high byte (no v_cvt_scalef32_pk_fp8_f16), "nofence" drops the sched_barrier pair around each
# bin's lo8 ring refill. dftx is the control (unchanged code).
# usage (through gpurun): bash tools/gpu_r06y.sh TAG
set -o pipefail
TAG=${1:-r06y}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out || exit 1
bash tools/ab_fp32.sh $TAG "dftp dftx" "" libbcfft_exp_nocvt.so libbcfft_exp_nofence.so
