#!/bin/bash
# Round 5: is the ramp (first ~200 batches 10-20 % slow) tied to the key-table footprint?
# Ramp windows after idle with 4,096 keys (43 GB of comb tables) vs 64 keys (0.7 GB), 3 streams.
set -o pipefail
out=gpurun_out/r05_tlb
mkdir -p $out
for rep in 1 2; do
  for nk in 64 4096; do
    timeout -k 10 240 python -u tools/timed_region_probe.py --steps 20 200 --reps 2 --streams 3 --ramp 400 --nkeys $nk \
      > $out/k${nk}_$rep.jsonl 2> $out/k${nk}_$rep.err || { tail -5 $out/k${nk}_$rep.err; exit 1; }
    python3 - $out/k${nk}_$rep.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    if "ramp_after_idle_s" in d:
        print("nkeys", d["nkeys"], "idle", d["ramp_after_idle_s"], "win20", d["window20_ms_per_step"][:8], "...", d["window20_ms_per_step"][-3:])
    else:
        print("nkeys region", d["steps"], d["rep"], d["host_ms_per_step"], d.get("steady_ms_per_step"))
PY
  done
done
