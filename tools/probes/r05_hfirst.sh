#!/bin/bash
# Round 5: the driver's 20-step headline timed right after the key-table build (--headline-first 1)
# or after the PCIe leg (0); then the split tree finish A/B (r05_split.sh).
set -o pipefail
out=gpurun_out/r05_hfirst
mkdir -p $out
for rep in 1 2 3; do
  for hf in 1 0; do
    timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu --latency-runs 0 \
      --headline-first $hf > $out/hf${hf}_$rep.json 2> $out/hf${hf}_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$out/hf${hf}_$rep.json'));print('headline_first $hf rep $rep', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d['pcie_inclusive_value']/1e6,1), d.get('step_spread_ms'), d.get('sclk_mhz'))"
  done
done
bash tools/probes/r05_split.sh
