#!/bin/bash
# Round 5: the pair ladder's first addition as a point set (1 M instead of 7): parity, then the
# headline at 2 / 3 streams (tree finish 64 x 2), then the config #3 knobs (r05_mixed2.sh).
set -o pipefail
out=gpurun_out/r05_first
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_ed25519_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 \
  --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
  for st in 2 3; do
    CBFT_FINISH_TREE_BLOCK=64 timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-extras --no-cpu \
      --latency-runs 0 --streams $st > $out/st${st}_$rep.json 2> $out/st${st}_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$out/st${st}_$rep.json'));print('first-set streams $st rep $rep', round(d['value']/1e6,1), round(d['ms_per_step'],4), d.get('step_spread_ms'), d.get('sclk_mhz'), d['roofline']['stage_ms_pipelined'], d['roofline']['stage_ms_isolated'])"
  done
done
bash tools/probes/r05_mixed2.sh
