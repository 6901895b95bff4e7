#!/bin/bash
# Round 5: parity of the quad comb's first point set (small batches, quad ladder), the lone-call /
# p50 path, then the stage-order A/B (r05_order.sh).
set -o pipefail
out=gpurun_out/r05_quad
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_ed25519_gpu.py tests/test_cpp_host.py -x -q --timeout 120 \
  --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 120 python -u tools/lone_probe.py > $out/lone.txt 2>&1 || { tail -20 $out/lone.txt; exit 1; }
tail -5 $out/lone.txt
bash tools/probes/r05_order.sh
