# HBM traffic of the fp32 headline (dftx) and the bf16 north star after the round-4 kernel changes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/pmc_groups.sh hs32 FETCH_SIZE WRITE_SIZE > gpurun_out/pmc_hs32.log 2>&1 &&
RUN="4096 4096 128 bf16 8192" bash tools/pmc_groups.sh hs16 FETCH_SIZE WRITE_SIZE > gpurun_out/pmc_hs16.log 2>&1 &&
python3 tools/pmc_traffic.py r04b 4096x4096_b128_n8192_fp32=gpurun_out/pmc_hs32@dftx 4096x4096_b128_n8192_bf16=gpurun_out/pmc_hs16@dft > gpurun_out/pmc_traffic_r04b.log 2>&1
