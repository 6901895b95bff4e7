cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT && \
RUNS="base@concord-bft_amd/libcbft_hipcrypto.so@2@1 ws4s2@build/lib_ws4.so@2@1 ws4s3@build/lib_ws4.so@3@1 ws4s4@build/lib_ws4.so@4@1 ws4s3o3@build/lib_ws4.so@3@3 ws4s3o0@build/lib_ws4.so@3@0 base2@concord-bft_amd/libcbft_hipcrypto.so@2@1 ws4s3b@build/lib_ws4.so@3@1" timeout -k 10 500 bash tools/gpu_devsweep.sh && \
(cd /tmp && CBFT_LIB=$R/build/lib_ws4.so NSTREAMS=3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace3" -o run -- python3 "$R/tools/dev_pipe_probe.py") > gpurun_out/trace3_probe.log 2>&1 && \
python3 tools/trace_timeline.py $(find gpurun_out/trace3 -name "*kernel_trace.csv" | head -1) ed25519_ --skip 60 --count 24
