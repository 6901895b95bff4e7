set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_ed25519_gpu.py tests/test_pipeline_gpu.py tests/test_cpp_host.py "tests/test_bls_gpu.py::test_keyset_rotation_per_checkpoint_window" -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_ed.log 2>&1 || { tail -30 gpurun_out/pytest_ed.log; exit 1; }
tail -1 gpurun_out/pytest_ed.log
for f in 2 3; do CBFT_ENGINE_INFLIGHT=$f timeout -k 10 120 tools/host_bench 64 2000 1024 16 > gpurun_out/host_bench_if$f.json || exit 1; python3 -c "
import json; d=json.load(open('gpurun_out/host_bench_if$f.json')); print('inflight $f', {k: (d[k]['verifies_per_s'], d[k]['p50_us'], d[k]['calls_per_batch']) for k in ('verify_mt','verifysig_mt','single','openssl_mt')})"; done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { tail -5 gpurun_out/bench_q.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_q.json')); print('bench', d['value'], d['device_resident_value'], d['p50_latency_ms_batch1k'], d['key_table_load_ms'])"
