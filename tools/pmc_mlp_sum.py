"""Sum the per-launch FETCH_SIZE (x2, the gfx950 correction of tools/pmc_traffic.py) and WRITE_SIZE
of the BC kernels of one MLP call (fused: bc_mlp_dmm_kernel; split: bc_forward_dmg_kernel +
bc_forward_dmk_kernel) from tools/pmc_mlp.sh's passes. usage: pmc_mlp_sum.py DIR [DIR ...]"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = ("bc_mlp_dmm_kernel", "bc_forward_dmg_kernel", "bc_forward_dmk_kernel")


def main():
    res = {}
    for d in sys.argv[1:]:
        acc = collections.defaultdict(list)
        for f in glob.glob(os.path.join(d, "g*", "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
                if k:
                    acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
        per = {}
        for (k, c), v in acc.items():
            per.setdefault(k, {})[c] = sum(v) / len(v)
        tot_r = sum(cs.get("FETCH_SIZE", 0.0) for cs in per.values()) * 1024 * 2
        tot_w = sum(cs.get("WRITE_SIZE", 0.0) for cs in per.values()) * 1024
        res[os.path.basename(d.rstrip("/"))] = {
            "kernels": {k: {"read_bytes_corrected": int(cs.get("FETCH_SIZE", 0.0) * 2048),
                            "write_bytes": int(cs.get("WRITE_SIZE", 0.0) * 1024)} for k, cs in per.items()},
            "read_bytes_per_mlp": int(tot_r), "write_bytes_per_mlp": int(tot_w),
            "hbm_bytes_per_mlp": int(tot_r + tot_w), "n_tokens": 8192,
            "x_plus_y_bytes": 2 * 8192 * 4096 * 2}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
