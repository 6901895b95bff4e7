#!/bin/bash
# A/B of the Ed25519 pipeline schedule: cross-batch stage order, finish batching, batches in flight.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
IFS=";" read -ra LIST <<< "${CFGS:-1 8 2;0 8 2;1 4 2;1 16 2;1 8 3}"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  CBFT_STAGE_ORDER=$1 CBFT_FINISH_BATCH=$2 timeout -k 10 120 python -u bench.py --steps 200 --warmup 10 --no-cpu --latency-runs 0 --no-extras --inflight $3 > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "fail $cfg"; tail -20 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print('order=$1 K=$2 inflight=$3', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step', d['roofline'].get('stage_ms'))" | tee -a gpurun_out/ab_summary.txt
done
