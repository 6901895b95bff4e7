#!/bin/bash
# RSA kernel A/B: parity tests under each kernel, then the quick timing (e = 65537 and 17).
set -o pipefail
mkdir -p gpurun_out
for k in pair fios; do
  CBFT_RSA_KERNEL=$k timeout -k 10 300 python -u -m pytest tests/test_rsa_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/rsa_test_$k.log 2>&1 || { echo "tests failed ($k)"; tail -30 gpurun_out/rsa_test_$k.log; exit 1; }
  echo "$k: $(tail -1 gpurun_out/rsa_test_$k.log)"
  for e in 65537 17; do
    CBFT_RSA_KERNEL=$k timeout -k 10 120 python -u tools/rsa_quick.py 65536 $e > gpurun_out/rsa_q_${k}_$e.log 2>&1 || { echo "timing failed"; tail -5 gpurun_out/rsa_q_${k}_$e.log; exit 1; }
    echo "$k: $(tail -1 gpurun_out/rsa_q_${k}_$e.log)"
  done
done
