#!/bin/bash
# Round 5: the driver's bench command on the current tree, then the share-verify form A/B at
# k = 683 (760 shares): CBFT_BLS_SHARE_WAVES = 2 (two-wave blocks, final exponentiation helper)
# against the default (one wave per share beyond 512 shares).
set -o pipefail
out=gpurun_out/r05_bench_bls
mkdir -p $out
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench20.json 2> $out/bench20.err \
  || { tail -5 $out/bench20.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench20.json'));print('bench20', round(d['value']/1e6,1), d['ms_per_step'], d.get('step_spread_ms'), d['mixed_config3'], d['bls_config4'])"
for rep in 1 2; do
  for w in 0 2; do
    CBFT_BLS_SHARE_WAVES=$w timeout -k 10 120 python -u tools/bls_probe.py --reps 10 > $out/w${w}_$rep.json 2> $out/w${w}_$rep.err \
      || { tail -5 $out/w${w}_$rep.err; exit 1; }
    echo "waves=$w $rep $(tail -1 $out/w${w}_$rep.json | cut -c1-200)"
  done
done
