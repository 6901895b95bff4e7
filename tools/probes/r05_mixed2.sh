#!/bin/bash
# Round 5: config #3 device-resident: the long-message kernel's group cap and issue priority,
# K1's priority (2 streams, early hash order).
set -o pipefail
out=gpurun_out/r05_mixed2
mkdir -p $out
timeout -k 10 200 python -u -m pytest tests/test_ed25519_gpu.py -x -q -k "sort or mixed or long" \
  --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -20 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
  for cfg in "192 0 0" "256 0 0" "192 0 1" "256 0 1" "256 1 1" "320 0 1"; do
    set -- $cfg
    CBFT_SHA_LONG_GROUPS=$1 CBFT_HASH_PRIO=$2 CBFT_HASH_LONG_PRIO=$3 timeout -k 10 120 python -u tools/mixed_probe.py \
      --steps 40 --mixed-streams 2 > $out/g$1_p$2_l$3_$rep.json 2> $out/g$1_p$2_l$3_$rep.err || exit 1
    echo "groups $1 prio $2 long_prio $3 rep $rep $(cat $out/g$1_p$2_l$3_$rep.json)"
  done
done
