set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ed25519_gpu.py tests/test_pipeline_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_kl.log 2>&1 || { tail -30 gpurun_out/pytest_kl.log; exit 1; }
tail -1 gpurun_out/pytest_kl.log
for v in new old; do
  lib=""; [ $v = old ] && lib=tools/variant_keyload_old.so
  CBFT_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kl_$v -o run -- python3 tools/ed_keyload_probe.py 4096 > gpurun_out/kl_$v.log 2>&1 || { tail -5 gpurun_out/kl_$v.log; exit 1; }
  grep "load 4096" gpurun_out/kl_$v.log
done
timeout -k 10 200 python3 -u tools/ed_keyload_probe.py 4096
