#!/bin/bash
# Disassemble the gfx950 code object of every product object file (llama-fft_amd/lib/obj/*.o,
# built by `make -C llama-fft_amd`) into OUTDIR/<tu>.s without addresses, and print their md5s.
# Two snapshots taken before and after a source edit that must not change the product's code
# (e.g. moving analysis scaffolding, bcfft_analysis.h) compare equal line for line.
# usage: tools/isa_snapshot.sh OUTDIR
out=${1:?usage: isa_snapshot.sh OUTDIR}; mkdir -p "$out"; llvm=/opt/rocm/lib/llvm/bin
tmp=$(mktemp -d)
for o in "$(dirname "$0")"/../llama-fft_amd/lib/obj/*.o; do
  n=$(basename "$o" .o)
  objcopy -O binary --only-section=.hip_fatbin "$o" "$tmp/fat_$n.bin" || exit 1
  $llvm/clang-offload-bundler --unbundle --type=o --input="$tmp/fat_$n.bin" \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$tmp/dev_$n.o" || exit 1
  $llvm/llvm-objdump -d --no-show-raw-insn "$tmp/dev_$n.o" | tail -n +3 | sed -E 's/^ *[0-9a-f]+:\s*//; s/\/\/ [0-9A-F]+://' > "$out/$n.s"
done
rm -rf "$tmp"
md5sum "$out"/*.s
