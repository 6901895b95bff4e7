#!/bin/bash
# BLS GPU tests, then the keyset A/B (tools/keys_ab.sh) over the given variants
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bls_gpu.py tests/test_relic_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bls.log 2>&1 || { tail -30 gpurun_out/pytest_bls.log; exit 1; }
tail -1 gpurun_out/pytest_bls.log
bash tools/keys_ab.sh "$@"
