#!/bin/bash
# Finish-kernel batching (signatures per shared inversion, $CBFT_FINISH_BATCH) in the device-resident
# pipeline: the committed library over 2 streams and a 4-work-slot build (build/lib_ws4.so) over 3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for fb in 2 4 8 16; do
  echo "== finish batch $fb"
  CBFT_FINISH_BATCH=$fb RUNS="base@concord-bft_amd/libcbft_hipcrypto.so@2@1 ws4s3@build/lib_ws4.so@3@1" \
    timeout -k 10 300 bash tools/gpu_devsweep.sh || exit 1
done
