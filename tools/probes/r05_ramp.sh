#!/bin/bash
# Round 5: does the pipeline speed up over its first batches after an idle period (clock ramp)?
# Then the phased pair ladder: parity + headline A/B against the unphased build of this tree.
set -o pipefail
out=gpurun_out/r05_ramp
mkdir -p $out
timeout -k 10 200 python -u tools/timed_region_probe.py --steps 20 --reps 1 --ramp 400 --streams 3 > $out/ramp.jsonl 2> $out/ramp.err || { tail -20 $out/ramp.err; exit 1; }
cat $out/ramp.jsonl
timeout -k 10 400 python -u -m pytest tests/test_ed25519_gpu.py -x -q -k "ladder or golden or full_size or fixed" --timeout 120 \
  --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
  for lib in phased unphased; do
    CBFT_LIB=$GRAFT_REPO_ROOT/build/lib_$lib.so CBFT_FINISH_TREE_BLOCK=64 timeout -k 10 200 python -u bench.py --steps 200 \
      --warmup 20 --no-extras --no-cpu --latency-runs 0 --streams 3 > $out/${lib}_$rep.json 2> $out/${lib}_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$out/${lib}_$rep.json'));print('$lib rep $rep', round(d['value']/1e6,1), round(d['ms_per_step'],4), d.get('step_spread_ms'), d['roofline']['stage_ms_pipelined'], d['roofline']['stage_ms_isolated'])"
  done
done
