#!/bin/bash
# usage: tools/pmc_groups.sh TAG "GROUP1" "GROUP2" ... ; env RUN="K M B IO N" (default north star)
# one rocprofv3 --pmc pass per group (each under its own kill timeout), then a per-kernel summary
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
RUN=${RUN:-"4096 4096 128 fp32 8192"}
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/g$i -o run -- \
      python3 tools/run_fwd.py $RUN 6 > $OUT/g$i.log 2>&1 || echo "group $i ($grp) failed rc=$?" >> $OUT/failures.txt
done
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/g*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        print(f"{k:40s} {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
PY
