"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc*/.../*counter_collection.csv) per kernel and
write the ladder's HBM traffic record bench.py reads (profiles/pmc_ladder.json).

HBM bytes per launch = FETCH_SIZE x 2 + WRITE_SIZE (KB -> B): the x2 is the gfx950 correction
for 16-B-per-lane reads from MI355X_MICROARCH.md's HBM/rocprofv3 section."""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(root):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{root}/pmc*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0]
            acc[name][r["Counter_Name"]].append((r.get("Dispatch_Id"), float(r["Counter_Value"])))
    out = {}
    for k, ctrs in acc.items():
        out[k] = {}
        for c, vals in ctrs.items():
            per = defaultdict(float)  # sum over XCD/SE instances within a dispatch
            for d, v in vals:
                per[d] += v
            out[k][c] = sum(per.values()) / len(per)
    return out


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    kernel = sys.argv[2] if len(sys.argv) > 2 else "ed25519_comb_ladder_kernel"
    extra = json.loads(sys.argv[3]) if len(sys.argv) > 3 else {}
    c = load(root)
    k = c[kernel]
    rec = {"kernel": kernel, **extra,
           "FETCH_SIZE_KB": k.get("FETCH_SIZE"), "WRITE_SIZE_KB": k.get("WRITE_SIZE"),
           "hbm_bytes_per_launch": (k["FETCH_SIZE"] * 2 + k["WRITE_SIZE"]) * 1024
           if "FETCH_SIZE" in k and "WRITE_SIZE" in k else None,
           "counters": c}
    if "SQ_INSTS_VALU" in k and "SQ_WAVES" in k:
        rec["valu_insts_per_wave"] = k["SQ_INSTS_VALU"] / k["SQ_WAVES"]
    json.dump(rec, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
