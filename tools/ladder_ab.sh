#!/bin/bash
# A/B of Ed25519 ladder variants: "label|env assignments" per entry of $CFGS (';'-separated).
# Each runs bench.py without extras; prints value, device-resident ceiling and stage times.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
IFS=";" read -ra LIST <<< "$CFGS"
for cfg in "${LIST[@]}"; do
  label=${cfg%%|*}; envs=${cfg#*|}
  env $envs timeout -k 10 150 python -u bench.py --steps 200 --warmup 10 --no-cpu --latency-runs 0 --no-extras > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "fail $label"; tail -20 gpurun_out/ab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab.json')); r=d['roofline']
print('$label', 'value %.1f M/s' % (d['value']/1e6), 'device %.1f M/s' % (r['device_resident_ceiling']/1e6),
      'iso', {k: round(v*1e3,1) for k,v in r['stage_ms_isolated'].items()}, 'pipe', {k: round(v*1e3,1) for k,v in r['stage_ms_pipelined'].items()})" | tee -a gpurun_out/ab_summary.txt
done
