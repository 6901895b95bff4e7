set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ed25519_gpu.py tests/test_pipeline_gpu.py tests/test_cpp_host.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_sm.log 2>&1 || { tail -30 gpurun_out/pytest_sm.log; exit 1; }
tail -1 gpurun_out/pytest_sm.log
CBFT_LIB=tools/variant_edphases.so timeout -k 10 120 python3 -u tools/ed_small_probe.py
for f in 3 4 6; do
  CBFT_ENGINE_INFLIGHT=$f timeout -k 10 120 tools/host_bench 64 2000 1024 16 > gpurun_out/hb2_f$f.json || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/hb2_f$f.json')); print('inflight $f', {k: (d[k]['verifies_per_s'], d[k]['p50_us'], d[k]['calls_per_batch']) for k in ('verify_mt','verifysig_mt','single','openssl_mt')})"
done
