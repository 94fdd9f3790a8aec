#!/bin/bash
# Round 6: what the precise engine's weight-residual stream costs. Two
# timing-only builds of bcfft_dm.hip (their dftp results are wrong by construction, so no parity
# run): "l1" reads one 1 KiB piece per wave for every (bin, K-step) (L1 hits: no L2 stream),
# "half" reads each piece pair's first piece twice (half the distinct bytes: an e2m1 image's
# stream). dftx is the control (its code is unchanged in both builds).
# usage (through gpurun): bash tools/gpu_r06r.sh TAG
set -o pipefail
TAG=${1:-r06r}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out || exit 1
bash tools/ab_fp32.sh $TAG "dftp dftx" "" libbcfft_exp_l1.so libbcfft_exp_half.so
