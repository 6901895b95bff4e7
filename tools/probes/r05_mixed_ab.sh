#!/bin/bash
# Round 5: config #3 (mixed 64..4,096-B messages) device-resident rate: streams x work slots x
# whether the next batch's hash waits for the long-message tail (CBFT_HASH_ORDER_EARLY).
set -o pipefail
out=gpurun_out/r05_mixed
mkdir -p $out
timeout -k 10 200 python -u -m pytest tests/test_ed25519_gpu.py -x -q -k "sort or mixed or device or long" \
  --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -20 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
  for cfg in "2 2 0" "2 2 1" "4 4 0" "4 4 1" "3 4 1"; do
    set -- $cfg
    CBFT_WORK_SLOTS=$2 CBFT_HASH_ORDER_EARLY=$3 timeout -k 10 120 python -u tools/mixed_probe.py --steps 40 \
      --mixed-streams $1 > $out/s$1_w$2_e$3_$rep.json 2> $out/s$1_w$2_e$3_$rep.err || exit 1
    cat $out/s$1_w$2_e$3_$rep.json
  done
done
