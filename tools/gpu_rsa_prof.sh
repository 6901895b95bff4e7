#!/bin/bash
# RSA kernel: rocprofv3 kernel stats of the quick timing run (e = 65537 client keys, 64K).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/rsaprof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/rsa_quick.py" 65536 65537 > "$GRAFT_REPO_ROOT/gpurun_out/rsaprof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/rsaprof.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"; tail -1 gpurun_out/rsaprof.log; find gpurun_out/rsaprof -name "*kernel_stats.csv"
