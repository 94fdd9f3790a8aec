#!/bin/bash
# Analysis builds of the precise engine (dftp) for 16-bit x, which the product refuses (DESIGN.md
# section 6b): a patched copy of bcfft_dm.hip routes mode 2 with bf16 / fp16 x and an fp32 output
# to bc_forward_dm_kernel<XT, true, true, false, EP, BM>, one library per residual-term set EP
# (1 stage-1 table residual, 2 weight residual, 4 stage-3 table residual). tools/dbg_ep9b.py then
# compares 16-bit x against fp32 x holding the same values, per input block.
# usage: tools/dbg_dftp16_build.sh [EP ...]   -> llama-fft_amd/lib/libbcfft_exp_x16_EP.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
[ "${BIAS16:-0}" = 1 ] || for ep in "${@:-1 2 4 7}"; do
  python3 - "$ROOT" "$ep" <<'PY'
import sys
root, ep = sys.argv[1], sys.argv[2]
s = open(f"{root}/llama-fft_amd/csrc/bcfft_dm.hip").read()
old = "  if (mode == 2 && yf32 && xdt == BCFFT_F32 && (bias_dt == BCFFT_NONE || bias_dt == BCFFT_F32)) {"
assert s.count(old) == 1
new = ("  if (mode == 2 && yf32 && xdt != BCFFT_F32 && (bias_dt == BCFFT_NONE || bias_dt == BCFFT_F32)) {\n"
       f"    if (xdt == BCFFT_BF16) launch_dm<BCFFT_BF16, true, true, false, {ep}, 1>(x, n, n_out, spec, bias, bias_dt, y, s);\n"
       f"    else launch_dm<BCFFT_F16, true, true, false, {ep}, 1>(x, n, n_out, spec, bias, bias_dt, y, s);\n"
       "    return true;\n  }\n" + old)
open(f"/tmp/bcfft_dm_x16_{ep}.hip", "w").write(s.replace(old, new))
PY
  "$ROOT/tools/exp_one.sh" "x16_$ep" bcfft_dm "" "/tmp/bcfft_dm_x16_$ep.hip"
done
# second family (BIAS16=1): fp32 x with a 16-bit bias, the precise engine's BM = 2 instantiation
# -> libbcfft_exp_b16_EP.so (tools/dbg_dftp_bias16.py)
if [ "${BIAS16:-0}" = 1 ]; then
  for ep in "${@:-1 2 4 7}"; do
    python3 - "$ROOT" "$ep" <<'PY'
import sys
root, ep = sys.argv[1], sys.argv[2]
s = open(f"{root}/llama-fft_amd/csrc/bcfft_dm.hip").read()
old = "  if (mode == 2 && yf32 && xdt == BCFFT_F32 && (bias_dt == BCFFT_NONE || bias_dt == BCFFT_F32)) {"
assert s.count(old) == 1
new = ("  if (mode == 2 && yf32 && xdt == BCFFT_F32 && (bias_dt == BCFFT_BF16 || bias_dt == BCFFT_F16)) {\n"
       f"    launch_dm<BCFFT_F32, true, true, false, {ep}, 2>(x, n, n_out, spec, bias, bias_dt, y, s);\n"
       "    return true;\n  }\n" + old)
open(f"/tmp/bcfft_dm_b16_{ep}.hip", "w").write(s.replace(old, new))
PY
    "$ROOT/tools/exp_one.sh" "b16_$ep" bcfft_dm "" "/tmp/bcfft_dm_b16_$ep.hip"
  done
fi
