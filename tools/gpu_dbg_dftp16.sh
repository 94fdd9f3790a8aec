# dftp with 16-bit x per residual-term set (tools/dbg_dftp16_build.sh libraries): tools/dbg_ep9b.py
# per library; the first failure ends the call.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/${1:-dftp16} || exit 1
for ep in ${EPS:-1 2 4 7}; do
  echo "== EP $ep"
  BCFFT_LIB_PATH=llama-fft_amd/lib/libbcfft_exp_x16_$ep.so timeout -k 10 120 python3 -u tools/dbg_ep9b.py 2>&1 | grep -v amdgpu.ids || exit 1
done | tee gpurun_out/${1:-dftp16}/dbg.txt
