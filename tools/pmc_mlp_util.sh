#!/bin/bash
# utilisation and L2 counters of the fused BC-MLP (bc_mlp_dmm_kernel) at N = 8192: one rocprofv3
# --pmc pass per group (kernel trace only beside it, each under its own kill timeout)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_mlp_util
mkdir -p $OUT
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
G2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
G3="SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_COEXEC_CYCLES"
G4="TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum"
i=0
for grp in "$G1" "$G2" "$G3" "$G4"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/g$i -o run -- \
      python3 tools/run_mlp.py 8192 fused 6 > $OUT/g$i.log 2>&1 || echo "group $i ($grp) failed rc=$?" >> $OUT/failures.txt
done
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/g*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "bc_mlp_dmm" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for c, v in sorted(acc.items()):
        print(f"bc_mlp_dmm_kernel {c:32s} {sum(v) / len(v):18.1f}  (n={len(v)})")
PY
cat $OUT/failures.txt 2>/dev/null
exit 0
