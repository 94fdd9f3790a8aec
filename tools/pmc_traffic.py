"""Per-launch HBM traffic of the BC forward kernels from rocprofv3 FETCH_SIZE / WRITE_SIZE passes
(tools/pmc_groups.sh output) -> profiles/pmc_traffic_<round>.json, read by bench.py's roofline.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts 64 B per 128-B memory-side
read request on gfx950, i.e. exactly half the bytes of a wide coalesced streaming read, so it
is doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores. Both are in KiB.
usage: python tools/pmc_traffic.py ROUND TAG=gpurun_out/pmc_DIR[@ALGO] [TAG=DIR[@ALGO] ...]
       TAG is bench.py's workload tag, e.g. 4096x4096_b128_n8192_fp32; ALGO the engine measured
       (bench.py matches it against the engine AUTO resolves to)"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("bc_mlp_dmm_kernel", "bc_forward_dm_kernel", "bc_forward_dm8_kernel", "bc_forward_dmk_kernel", "bc_forward_dm64_kernel",
           "bc_forward_dmg_kernel", "bc_forward_dm256_kernel", "bc_forward_dm256k_kernel", "bc_forward_dm64k_kernel", "bc_forward_dm64g_kernel", "bc_forward_dm256g_kernel",
           "bc_forward_stat_kernel", "bc_forward_mfma_kernel", "bc_forward_valu_kernel")


def collect(d):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "g*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
            if name:
                acc[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
    out = {}
    for (k, c), v in acc.items():
        out.setdefault(k, {})[c] = {"mean": sum(v) / len(v), "n": len(v)}
    return out


def main():
    rnd = sys.argv[1]
    res = {}
    for arg in sys.argv[2:]:
        tag, d = arg.split("=", 1)
        d, _, algo = d.partition("@")
        per = collect(d)
        for k, cs in per.items():
            if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
                continue
            fetch = cs["FETCH_SIZE"]["mean"] * 1024 * 2      # KiB, x2 gfx950 correction
            write = cs["WRITE_SIZE"]["mean"] * 1024
            res[tag] = {"kernel": k, "hbm_bytes_per_launch": int(fetch + write),
                        "read_bytes_corrected": int(fetch), "write_bytes": int(write),
                        "raw_FETCH_SIZE_KiB": cs["FETCH_SIZE"]["mean"],
                        "raw_WRITE_SIZE_KiB": cs["WRITE_SIZE"]["mean"],
                        "launches": cs["FETCH_SIZE"]["n"], "source": d}
            if algo:
                res[tag]["algo"] = algo
    path = os.path.join(ROOT, "profiles", f"pmc_traffic_{rnd}.json")
    json.dump(res, open(path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
