set -o pipefail
for f in 2 3 4; do CBFT_ENGINE_INFLIGHT=$f timeout -k 10 120 tools/host_bench 64 2000 1024 16 > gpurun_out/host_bench_if$f.json || exit 1; python3 -c "
import json; d=json.load(open('gpurun_out/host_bench_if$f.json')); print('inflight $f', {k: (d[k]['verifies_per_s'], d[k]['p50_us'], d[k]['calls_per_batch']) for k in ('verify_mt','single','openssl_mt')})"; done
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py tests/test_ed25519_gpu.py tests/test_cpp_host.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -1
