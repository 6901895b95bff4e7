set -o pipefail
export TMPDIR=/tmp
CBFT_ENGINE_INFLIGHT=8 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d gpurun_out/rq8 -o run -- tools/host_bench 64 500 1024 16 > gpurun_out/rq8.json 2> gpurun_out/rq8.err || { tail -5 gpurun_out/rq8.err; exit 1; }
