#!/bin/bash
# keyset-load A/B: kernel stats of tools/bls_probe.py per library variant ($@: .so names)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in "$@"; do
  mkdir -p "$R/gpurun_out/keysab/$v"
  cd /tmp
  CBFT_LIB=$R/concord-bft_amd/$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/keysab/$v" -o run -- python3 "$R/tools/bls_probe.py" --reps 2 > "$R/gpurun_out/keysab/$v/probe.json" 2> "$R/gpurun_out/keysab/$v/err.txt" || { echo "$v failed"; tail -5 "$R/gpurun_out/keysab/$v/err.txt"; exit 1; }
  echo "$v $(cat $R/gpurun_out/keysab/$v/probe.json)"
done
