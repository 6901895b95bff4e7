#!/bin/bash
# Round 5: the split tree finish (block trees through HBM, one lane per root inversion) against the
# one-launch tree finish, headline at 3 streams, plus parity of every finish form.
set -o pipefail
out=gpurun_out/r05_split
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_ed25519_gpu.py -x -q -k "finish or full_size or fixed or two_streams" \
  --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
  for cfg in "0 64" "1 64" "1 128"; do
    set -- $cfg
    CBFT_FINISH_SPLIT=$1 CBFT_FINISH_TREE_BLOCK=$2 timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 \
      --no-extras --no-cpu --latency-runs 0 > $out/s$1_t$2_$rep.json 2> $out/s$1_t$2_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$out/s$1_t$2_$rep.json'));print('split $1 tree $2 rep $rep', round(d['value']/1e6,1), round(d['ms_per_step'],4), d.get('step_spread_ms'), d['roofline']['stage_ms_pipelined'], d['roofline']['stage_ms_isolated'])"
  done
done
