# dm64k two-group workgroups: parity, interleaved A/B against the one-group build, then HBM traffic
# (FETCH_SIZE / WRITE_SIZE passes) of both at 11008 -> 4096, b = 64, bf16, N = 8192.
TAG=${1:-r06e}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
REPS=3 bash tools/gpu_ab_dm64k.sh $TAG libbcfft.so ${LIBB:-libbcfft_exp_np.so} || exit 1
export TMPDIR=/tmp
for lib in libbcfft.so ${LIBB:-libbcfft_exp_np.so}; do
  for grp in FETCH_SIZE WRITE_SIZE; do
    BCFFT_LIB_PATH=llama-fft_amd/lib/$lib timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
      -d gpurun_out/$TAG/pmc_${lib%.so}/g_$grp -o run -- python3 tools/run_fwd.py 11008 4096 64 bf16 8192 6 \
      > gpurun_out/$TAG/pmc_${lib%.so}_$grp.log 2>&1 || exit 1
  done
done
python3 - gpurun_out/$TAG <<'PY'
import csv, collections, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/pmc_*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "dm64k" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for c, v in acc.items():
        print(f.split("/")[-4] if False else f.replace(sys.argv[1], "")[:40], c, f"{sum(v)/len(v):.1f} KiB", len(v))
PY
