#!/bin/bash
# Round 5: pair-ladder carry passes: Y - X without a carry (CBFT_LADDER_SUBNC) and D + C lazy
# (CBFT_LADDER_LAZYSUM), default = both; subnc = SUBNC only; base = neither.  Ed25519 GPU tests on
# the default build, then interleaved isolated-stage probes and 100-step benches.
set -o pipefail
out=gpurun_out/r05_ladder_carries
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_ed25519_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 \
  --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
LIBS="both=default subnc=$PWD/build/lib_subnc.so base=$PWD/build/lib_base.so" ROUNDS=3 bash tools/ab_libs.sh || exit 1
