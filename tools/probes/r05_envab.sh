#!/bin/bash
# Round 5: environment-knob A/B on the default library: isolated stage times (tools/ladder_probe.py)
# and the headline at 20 and 200 steps, interleaved.  VARIANTS="label=ENV=V,ENV=V label=..." (a
# bare label = no variables), OUT=dir under gpurun_out.
set -o pipefail
out=gpurun_out/${OUT:-r05_envab}
mkdir -p $out
for rep in 1 2; do
  for lv in $VARIANTS; do
    label=${lv%%=*}; envs=""
    [[ $lv == *=* ]] && envs=$(echo "${lv#*=}" | tr ',' ' ')
    env $envs timeout -k 10 200 python -u tools/ladder_probe.py --reps 10 > $out/probe_${label}_$rep.json 2> $out/probe_${label}_$rep.err \
      || { tail -5 $out/probe_${label}_$rep.err; exit 1; }
    for st in 20 200; do
      env $envs timeout -k 10 200 python -u bench.py --steps $st --warmup 5 --no-extras --no-cpu --latency-runs 0 \
        > $out/b${st}_${label}_$rep.json 2> $out/b${st}_${label}_$rep.err || { tail -5 $out/b${st}_${label}_$rep.err; exit 1; }
    done
    python3 - $out $label $rep <<'PY'
import json, sys
o, v, r = sys.argv[1:]
p = json.loads(open(f"{o}/probe_{v}_{r}.json").read().strip().splitlines()[-1])
b20 = json.load(open(f"{o}/b20_{v}_{r}.json")); b200 = json.load(open(f"{o}/b200_{v}_{r}.json"))
print(v, r, "isolated", p["us"], "| 20 steps", round(b20["value"] / 1e6, 1), "| 200 steps", round(b200["value"] / 1e6, 1),
      b200["roofline"].get("stage_ms_pipelined"))
PY
  done
done
