#!/bin/bash
# rocprofv3 kernel stats of the BLS config #4 probe (tools/bls_probe.py) -> gpurun_out/blsprof/
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/blsprof
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/blsprof/trace" -o run -- python3 "$R/tools/bls_probe.py" > "$R/gpurun_out/blsprof/probe.json" 2> "$R/gpurun_out/blsprof/trace.err" || { echo trace failed; tail -20 "$R/gpurun_out/blsprof/trace.err"; exit 1; }
cat "$R/gpurun_out/blsprof/probe.json"
f=$(find "$R/gpurun_out/blsprof/trace" -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | cut -c1-150
