#!/bin/bash
# Round 5: SHA-512 bitop3 results pinned as 64-bit register pairs (CBFT_SHA_PAIR_PIN): Ed25519 GPU
# tests on the default build, then interleaved A/B against build/lib_nopin.so (headline + config #3).
set -o pipefail
out=gpurun_out/r05_sha_pin
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_ed25519_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 \
  --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
LIBS="pin=default nopin=$PWD/build/lib_nopin.so" ROUNDS=3 bash tools/ab_libs.sh || exit 1
LIBS="pin=default nopin=$PWD/build/lib_nopin.so" ROUNDS=2 MODE=mixed bash tools/ab_libs.sh || exit 1
