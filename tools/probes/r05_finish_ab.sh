#!/bin/bash
# Round 5: the tree finish (one inversion per 512-lane block) against the round-4 per-lane
# Montgomery finish (CBFT_FINISH_BATCH=2): GPU parity of the Ed25519 paths, then the headline
# bench at the driver's 20 steps and A/B at 200 steps (no side measurements).
set -o pipefail
out=gpurun_out/r05_ab
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_ed25519_gpu.py tests/test_pipeline_gpu.py -x -q \
  --timeout 120 --timeout-method thread > $out/pytest_ed.log 2>&1 || { tail -20 $out/pytest_ed.log; exit 1; }
tail -2 $out/pytest_ed.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/bench20.json 2> $out/bench20.err || exit 1
python3 -c "import json;d=json.load(open('$out/bench20.json'));print('driver-like', d['value']/1e6, d['ms_per_step'], d.get('step_spread_ms'), d.get('sclk_mhz'), d['roofline']['stage_ms_pipelined'], d['roofline']['stage_ms_isolated'])"
for rep in 1 2; do
  for fb in 2 -2; do
    CBFT_FINISH_BATCH=$fb timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-extras --no-cpu \
      --latency-runs 0 > $out/fb${fb}_$rep.json 2> $out/fb${fb}_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$out/fb${fb}_$rep.json'));print('finish $fb rep $rep', round(d['value']/1e6,1), round(d['ms_per_step'],4), d.get('step_spread_ms'), d.get('sclk_mhz'), d['roofline']['stage_ms_pipelined'], d['roofline']['stage_ms_isolated'])"
  done
done
