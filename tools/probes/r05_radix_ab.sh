#!/bin/bash
# Round 5: 15 additions per pair lane instead of 16: key comb radix 2^14 (19 positions, 20.9 MB per
# key, 86 GB at 4,096 keys) with B's comb at radix 2^24 (11 positions, 11.8 GB), against the
# default radix 2^13 keys + 2^22 B (20 + 12 positions).  200-step headline, no side legs.
set -o pipefail
out=gpurun_out/r05_radix
mkdir -p $out
for rep in 1 2; do
  for cfg in "13 22" "14 24" "14 22"; do
    set -- $cfg
    CBFT_COMB_BUDGET_GB=120 CBFT_B_RADIX=$2 timeout -k 10 240 python -u bench.py --steps 200 --warmup 20 --no-extras \
      --no-cpu --latency-runs 0 --comb-radix $1 > $out/k$1_b$2_$rep.json 2> $out/k$1_b$2_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$out/k$1_b$2_$rep.json'));print('key $1 B $2 rep $rep', round(d['value']/1e6,1), round(d['ms_per_step'],4), d.get('step_spread_ms'), d.get('sclk_mhz'), d['roofline']['stage_ms_pipelined'], d['key_table_load_ms'])"
  done
done
