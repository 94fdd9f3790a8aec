# round-4 counter passes: the one-launch MLP's HBM traffic after the stream policy, config 2's
# (dmg) traffic, and config 1's (stationary kernel, b = 64, N = 128 fp32) utilisation groups
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/pmc_mlp.sh > gpurun_out/pmc_mlp_r04.log 2>&1 || exit 1
for grp in FETCH_SIZE WRITE_SIZE; do
  mkdir -p gpurun_out/pmc_cfg2/$grp
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_cfg2/$grp -o run -- \
      python3 tools/run_fwd.py 4096 11008 128 bf16 8192 6 > gpurun_out/pmc_cfg2/$grp.log 2>&1 || exit 1
done
bash tools/pmc.sh cfg1 4096 4096 64 fp32 128 > gpurun_out/pmc_cfg1.log 2>&1
