#!/bin/bash
# Round 5: the driver's 20-step headline under each stage order (3 streams), then the ramp trace.
set -o pipefail
out=gpurun_out/r05_order20
mkdir -p $out
for rep in 1 2 3; do
  for so in 1 0 2; do
    CBFT_STAGE_ORDER=$so timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu \
      --latency-runs 0 > $out/so${so}_$rep.json 2> $out/so${so}_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$out/so${so}_$rep.json'));print('order $so rep $rep', round(d['value']/1e6,1), round(d['ms_per_step'],4), d.get('step_spread_ms'), d.get('sclk_mhz'))"
  done
done
timeout -k 10 120 python -u tools/mixed_probe.py --steps 40 > $out/mixed_default.json 2>&1 || exit 1
echo "config3 default $(cat $out/mixed_default.json)"
bash tools/probes/r05_ramp_trace.sh
