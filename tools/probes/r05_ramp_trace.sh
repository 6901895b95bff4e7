#!/bin/bash
# Round 5: kernel trace of the ramp (400 batches after 1 s idle, 3 streams): per-kernel durations
# and gaps in the first 40 batches against batches 300-340.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r05_ramp_trace
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $out/t -o run -- python3 $R/tools/timed_region_probe.py \
  --steps 20 --reps 1 --ramp 400 --streams 3 > $out/probe.out 2>&1 || { tail -20 $out/probe.out; exit 1; }
f=$(find $out/t -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, statistics
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "ed25519" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
lad = [r for r in rows if "comb2_ladder" in r["Kernel_Name"]]
# the ramp run after 1 s idle: find the first ladder after a > 0.5 s gap
starts = [int(r["Start_Timestamp"]) for r in lad]
k0 = next(i for i in range(1, len(starts)) if starts[i] - starts[i - 1] > 5e8)
seg = lad[k0:k0 + 400]
def dur(r): return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for name in ("comb2_ladder", "hash_kernel", "finish_tree"):
    ks = [r for r in rows if name in r["Kernel_Name"] and int(r["Start_Timestamp"]) >= int(seg[0]["Start_Timestamp"]) - 300000]
    ks = ks[:400]
    print(name, "first 40 mean us", round(statistics.mean(dur(r) for r in ks[:40]), 1),
          "batches 300-340", round(statistics.mean(dur(r) for r in ks[300:340]), 1))
st = [int(r["Start_Timestamp"]) for r in seg]
print("ladder start-to-start us: first 40", round((st[40] - st[0]) / 40e3, 1), "300-340", round((st[340] - st[300]) / 40e3, 1))
PY
