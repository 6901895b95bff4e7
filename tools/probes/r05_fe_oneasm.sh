#!/bin/bash
# Round 5: one asm statement per field multiply (CBFT_FE_ONEASM) vs one per column: Ed25519 GPU
# tests on the default build, then interleaved A/B against build/lib_colasm.so (headline + config #3).
set -o pipefail
out=gpurun_out/r05_fe_oneasm
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_ed25519_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 \
  --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
LIBS="oneasm=default colasm=$PWD/build/lib_colasm.so" ROUNDS=3 bash tools/ab_libs.sh || exit 1
LIBS="oneasm=default colasm=$PWD/build/lib_colasm.so" ROUNDS=2 MODE=mixed bash tools/ab_libs.sh || exit 1
