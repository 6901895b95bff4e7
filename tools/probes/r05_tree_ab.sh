#!/bin/bash
# Round 5: tree-finish block sizes against the per-lane finish (K = 2) in the headline pipeline
# (2 and 3 streams), then where the contract's timed region spends its time (20 / 200 steps).
set -o pipefail
out=gpurun_out/r05_tree
mkdir -p $out
timeout -k 10 200 python -u -m pytest tests/test_ed25519_gpu.py -x -q -k "finish" --timeout 120 \
  --timeout-method thread > $out/pytest.log 2>&1 || { tail -20 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
  for cfg in "2 2 128" "2 -2 128" "2 -2 64" "2 -4 64" "3 2 128" "3 -2 128"; do
    set -- $cfg
    CBFT_FINISH_BATCH=$2 CBFT_FINISH_TREE_BLOCK=$3 timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 \
      --no-extras --no-cpu --latency-runs 0 --streams $1 > $out/st$1_fb$2_t$3_$rep.json 2> $out/st$1_fb$2_t$3_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$out/st$1_fb$2_t$3_$rep.json'));print('streams $1 finish $2 tree $3 rep $rep', round(d['value']/1e6,1), round(d['ms_per_step'],4), d.get('step_spread_ms'), d.get('sclk_mhz'), d['roofline']['stage_ms_pipelined'])"
  done
done
CBFT_FINISH_BATCH=2 timeout -k 10 200 python -u tools/timed_region_probe.py --steps 20 200 --reps 3 > $out/timed_fb2.jsonl 2> $out/timed_fb2.err || exit 1
cat $out/timed_fb2.jsonl
CBFT_FINISH_BATCH=2 timeout -k 10 200 python -u tools/timed_region_probe.py --steps 20 200 --reps 2 --events 0 > $out/timed_fb2_noev.jsonl 2> $out/timed_fb2_noev.err || exit 1
cat $out/timed_fb2_noev.jsonl
