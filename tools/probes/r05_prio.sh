#!/bin/bash
# Round 5: pair-ladder issue priority by progress (CBFT_LADDER_PRIO): the per-wave end-time
# spread with it (stamps build), then isolated ladder time and the headline at 20 and 200 steps,
# interleaved default / prio.
set -o pipefail
out=gpurun_out/r05_prio
mkdir -p $out
CBFT_LIB=$PWD/build/lib_priostamps.so timeout -k 10 300 python -u tools/ladder_probe.py --reps 3 --nkeys 4096 \
  > $out/stamps.txt 2>&1 || { tail -5 $out/stamps.txt; exit 1; }
grep "comb2 ladder" $out/stamps.txt | tail -2
for rep in 1 2; do
  for v in default prio; do
    lib=$PWD/concord-bft_amd/libcbft_hipcrypto.so
    [ $v = default ] || lib=$PWD/build/lib_$v.so
    CBFT_LIB=$lib timeout -k 10 200 python -u tools/ladder_probe.py --reps 10 > $out/probe_${v}_$rep.json 2> $out/probe_${v}_$rep.err \
      || { tail -5 $out/probe_${v}_$rep.err; exit 1; }
    for st in 20 200; do
      CBFT_LIB=$lib timeout -k 10 200 python -u bench.py --steps $st --warmup 5 --no-extras --no-cpu --latency-runs 0 \
        > $out/b${st}_${v}_$rep.json 2> $out/b${st}_${v}_$rep.err || { tail -5 $out/b${st}_${v}_$rep.err; exit 1; }
    done
    python3 - $out $v $rep <<'PY'
import json, sys
o, v, r = sys.argv[1:]
p = json.loads(open(f"{o}/probe_{v}_{r}.json").read().strip().splitlines()[-1])
b20 = json.load(open(f"{o}/b20_{v}_{r}.json")); b200 = json.load(open(f"{o}/b200_{v}_{r}.json"))
print(v, r, "isolated", p["us"], "| 20 steps", round(b20["value"] / 1e6, 1), "| 200 steps", round(b200["value"] / 1e6, 1),
      b200["roofline"].get("stage_ms_pipelined"))
PY
  done
done
