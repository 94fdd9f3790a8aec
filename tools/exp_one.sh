#!/bin/bash
# Experiment library from the product objects with ONE translation unit rebuilt under extra defines:
# tools/exp_one.sh NAME SRC "DEFS" [FILE] -> llama-fft_amd/lib/libbcfft_exp_NAME.so (A/B and stamps
# builds of a single kernel without recompiling the others; FILE: another version of csrc/SRC.hip,
# e.g. from `git show`; run `make -C llama-fft_amd` first).
set -e
NAME=$1; SRC=$2; DEFS=$3; FILE=$4
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$ROOT/llama-fft_amd/lib/obj
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$ROOT/include -ffp-contract=fast -fno-slp-vectorize"
mkdir -p /tmp/exp_$NAME
if [ -n "$FILE" ]; then
  cp "$FILE" $ROOT/llama-fft_amd/csrc/.exp_$NAME.hip
  /opt/rocm/bin/hipcc $FLAGS $DEFS -c $ROOT/llama-fft_amd/csrc/.exp_$NAME.hip -o /tmp/exp_$NAME/$SRC.o
  rm -f $ROOT/llama-fft_amd/csrc/.exp_$NAME.hip
else
  /opt/rocm/bin/hipcc $FLAGS $DEFS -c $ROOT/llama-fft_amd/csrc/$SRC.hip -o /tmp/exp_$NAME/$SRC.o
fi
OBJS=$(ls $OBJ/*.o | grep -v "/$SRC.o$")
/opt/rocm/bin/hipcc $FLAGS -shared $OBJS /tmp/exp_$NAME/$SRC.o -o $ROOT/llama-fft_amd/lib/libbcfft_exp_$NAME.so
echo "built lib/libbcfft_exp_$NAME.so"
