#!/bin/bash
# A/B timing of experiment builds of the streamed-weight DFT kernel (bcfft_dmk.hip) in one GPU
# session. Build here: tools/ab_dmk.sh build NAME "DEFS" ... ; run on the box: tools/ab_dmk.sh run NAME ...
# ("" = the product library). Each variant links the product objects with a variant dmk object.
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
LIB=$ROOT/llama-fft_amd/lib
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$ROOT/include -ffp-contract=fast -fno-slp-vectorize"
if [ "$1" = build ]; then
  shift
  while [ $# -ge 2 ]; do
    NAME=$1; DEFS=$2; shift 2
    ( /opt/rocm/bin/hipcc $FLAGS $DEFS -c $ROOT/llama-fft_amd/csrc/bcfft_dmk.hip -o $LIB/obj/exp_dmk_$NAME.o &&
      /opt/rocm/bin/hipcc $FLAGS -shared $(ls $LIB/obj/*.o | grep -v "/exp_" | grep -v "bcfft_dmk.o") $LIB/obj/exp_dmk_$NAME.o \
        -o $LIB/libbcfft_exp_$NAME.so && echo built $NAME ) &
  done
  wait
  exit 0
fi
shift
mkdir -p $ROOT/gpurun_out
for round in 1 2; do
  for L in "$@"; do
    P=$LIB/libbcfft.so; [ -n "$L" ] && P=$LIB/libbcfft_exp_$L.so
    echo "== ${L:-product} round $round"
    BCFFT_LIB_PATH=$P timeout -k 10 120 python3 -u $ROOT/tools/time_algos.py dft --down2 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
