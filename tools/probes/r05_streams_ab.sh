#!/bin/bash
# Round 5: headline device-resident pipeline, streams x finish form (200 steps, no side legs),
# then the config #3 A/B (tools/probes/r05_mixed_ab.sh).
set -o pipefail
out=gpurun_out/r05_streams
mkdir -p $out
for rep in 1 2; do
  for cfg in "2 -2" "3 -2" "4 -2" "3 2" "2 2"; do
    set -- $cfg
    CBFT_FINISH_BATCH=$2 timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-extras --no-cpu \
      --latency-runs 0 --streams $1 > $out/st$1_fb$2_$rep.json 2> $out/st$1_fb$2_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$out/st$1_fb$2_$rep.json'));print('streams $1 finish $2 rep $rep', round(d['value']/1e6,1), round(d['ms_per_step'],4), d.get('step_spread_ms'), d.get('sclk_mhz'), d['roofline']['stage_ms_pipelined'])"
  done
done
bash tools/probes/r05_mixed_ab.sh
