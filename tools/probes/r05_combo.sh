#!/bin/bash
# Round 5: headline pipeline combinations (200 steps, no side legs): streams x tree-finish block /
# signatures per lane x stage order; then 15 additions per pair lane (key radix 14 + B radix 24).
set -o pipefail
out=gpurun_out/r05_combo
mkdir -p $out
run() {  # tag streams finish tree order [extra env...]
  local tag=$1 st=$2 fb=$3 tb=$4 so=$5; shift 5
  env CBFT_FINISH_BATCH=$fb CBFT_FINISH_TREE_BLOCK=$tb CBFT_STAGE_ORDER=$so "$@" timeout -k 10 200 python -u bench.py \
    --steps 200 --warmup 20 --no-extras --no-cpu --latency-runs 0 --streams $st --comb-radix ${RADIX:-13} > $out/$tag.json 2> $out/$tag.err || return 1
  python3 -c "import json;d=json.load(open('$out/$tag.json'));print('$tag', round(d['value']/1e6,1), round(d['ms_per_step'],4), d.get('step_spread_ms'), d.get('sclk_mhz'), d['roofline']['stage_ms_pipelined'])"
}
for rep in 1 2; do
  run st2_t64k2_$rep 2 -2 64 1 || exit 1
  run st3_t64k2_$rep 3 -2 64 1 || exit 1
  run st3_t64k1_$rep 3 -1 64 1 || exit 1
  run st2_t64k1_$rep 2 -1 64 1 || exit 1
  run st4_t64k2_$rep 4 -2 64 1 || exit 1
  run st3_t64k2_noorder_$rep 3 -2 64 0 || exit 1
  run st3_t128k2_$rep 3 -2 128 1 || exit 1
done
for rep in 1 2; do
  RADIX=14 run st3_k14b24_$rep 3 -2 64 1 CBFT_COMB_BUDGET_GB=120 CBFT_B_RADIX=24 || exit 1
done
