set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ed25519_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { tail -30 gpurun_out/pytest_ab.log; exit 1; }
tail -1 gpurun_out/pytest_ab.log
for rep in 1 2; do for v in new old; do
  lib=""; [ $v = old ] && lib=tools/variant_old.so
  CBFT_LIB=$lib timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-extras --no-cpu > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_$v.json')); r=d['roofline']; print('$v', round(d['value']/1e6,1), round(d['device_resident_value']/1e6,1), r.get('stage_ms_isolated'), r.get('stage_ms_pipelined'))"
done; done
