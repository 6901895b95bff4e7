#!/bin/bash
# A/B of the GPU-only ordering events without the system-scope fence (build/lib_nofence.so) against
# the committed library: bench.py headline (tools/ab_libs.sh), the device pipeline probe, and a
# kernel trace of the variant's two-stream pipeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
LIBS="base=default nofence=build/lib_nofence.so" ROUNDS=3 bash tools/ab_libs.sh || exit 1
RUNS="base@concord-bft_amd/libcbft_hipcrypto.so@2@1 nofence@build/lib_nofence.so@2@1 base2@concord-bft_amd/libcbft_hipcrypto.so@2@1 nofence2@build/lib_nofence.so@2@1" \
  timeout -k 10 300 bash tools/gpu_devsweep.sh || exit 1
(cd /tmp && CBFT_LIB=$R/build/lib_nofence.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace_nf" -o run \
  -- python3 "$R/tools/dev_pipe_probe.py") > gpurun_out/trace_nf_probe.log 2>&1 || { tail -20 gpurun_out/trace_nf_probe.log; exit 1; }
python3 tools/trace_timeline.py $(find gpurun_out/trace_nf -name "*kernel_trace.csv" | head -1) ed25519_ --skip 60 --count 12
