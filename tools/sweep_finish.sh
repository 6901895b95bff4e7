#!/bin/bash
# Sweep the batched-finish width and in-flight batches (one GPU call); prints one line per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for fb in ${FB_LIST:-1 2 4 8 16}; do
  for inf in ${INF_LIST:-1 2 3}; do
    CBFT_FINISH_BATCH=$fb timeout -k 10 120 python -u bench.py --steps 40 --no-cpu --latency-runs 0 --no-extras --inflight $inf \
      > gpurun_out/sw_${fb}_${inf}.json 2> gpurun_out/sw_${fb}_${inf}.err || { echo "fb=$fb inf=$inf failed"; tail -5 gpurun_out/sw_${fb}_${inf}.err; exit 1; }
    python -c "import json,sys; r=json.load(open('gpurun_out/sw_${fb}_${inf}.json')); print('fb=$fb inf=$inf', round(r['value']/1e6,1), 'M/s', {k: round(v*1e3,1) for k,v in r['roofline']['stage_ms'].items()})"
  done
done
