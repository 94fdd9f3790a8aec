# dftp analysis builds (tools/dbg_dftp16_build.sh): 16-bit x per residual-term set EP
# (tools/dbg_ep9b.py), then fp32 x with a 16-bit bias per EP (tools/dbg_dftp_bias16.py, BIAS16=1
# builds). The first failure ends the call.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/${1:-dftp16} || exit 1
{
echo "== probe: MFMA SrcC chains across opcodes"
timeout -k 10 30 tools/probe/srcc || exit 1
for ep in ${EPS:-1 2 4 7}; do
  echo "== 16-bit x, EP $ep"
  BCFFT_LIB_PATH=llama-fft_amd/lib/libbcfft_exp_x16_$ep.so timeout -k 10 120 python3 -u tools/dbg_ep9b.py 2>&1 | grep -v amdgpu.ids || exit 1
done
for ep in ${BEPS:-}; do
  echo "== fp32 x, 16-bit bias, EP $ep"
  BCFFT_LIB_PATH=llama-fft_amd/lib/libbcfft_exp_b16_$ep.so timeout -k 10 120 python3 -u tools/dbg_dftp_bias16.py 2>&1 | grep -v amdgpu.ids || exit 1
done
} | tee gpurun_out/${1:-dftp16}/dbg.txt
