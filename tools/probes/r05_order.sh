#!/bin/bash
# Round 5: cross-batch stage order (1 = hash after hash and ladder after ladder, 2 = ladders only,
# 3 = hashes only, 0 = none) for the headline (3 streams) and config #3 (4 streams).
set -o pipefail
out=gpurun_out/r05_order
mkdir -p $out
for rep in 1 2; do
  for so in 1 2 0; do
    CBFT_STAGE_ORDER=$so timeout -k 10 120 python -u tools/mixed_probe.py --steps 40 --mixed-streams 4 \
      > $out/mixed_so${so}_$rep.json 2> $out/mixed_so${so}_$rep.err || exit 1
    echo "config3 order $so rep $rep $(cat $out/mixed_so${so}_$rep.json)"
    CBFT_STAGE_ORDER=$so timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-extras --no-cpu \
      --latency-runs 0 > $out/head_so${so}_$rep.json 2> $out/head_so${so}_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$out/head_so${so}_$rep.json'));print('headline order $so rep $rep', round(d['value']/1e6,1), round(d['ms_per_step'],4), d.get('step_spread_ms'), d['roofline']['stage_ms_pipelined'])"
  done
done
