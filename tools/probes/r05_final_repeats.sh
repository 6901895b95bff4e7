#!/bin/bash
# Round 5: the driver's command three times back to back on one box (final tree), value + GFX clock.
set -o pipefail
out=gpurun_out/r05_final_repeats
mkdir -p $out
for r in 1 2 3; do
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench20_$r.json 2> $out/bench20_$r.err \
    || { tail -20 $out/bench20_$r.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], round(d['value']/1e6,1), d['ms_per_step'], d['sclk_mhz'], d['step_spread_ms'], round(d['mixed_config3']['device_resident_value']/1e6,1), d['bls_config4']['share_verify_ms'], d['bls_config4']['verify_ms'], d['bls_config4']['certificate_fused_ms'])" $out/bench20_$r.json $r
done
