set -o pipefail
export TMPDIR=/tmp
for so in 1 0 2; do
  CBFT_STAGE_ORDER=$so timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-extras --no-cpu --latency-runs 0 > gpurun_out/so_$so.json 2> gpurun_out/so_$so.err || { tail -5 gpurun_out/so_$so.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/so_$so.json')); r=d['roofline']; print('stage_order $so', round(d['value']/1e6,1), round(d['device_resident_value']/1e6,1), r.get('stage_ms_pipelined'))"
done
