# the driver's bench command on the current tree (N = 1), its line and detail record under gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-x}
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench_$tag.json 2> gpurun_out/r06_bench_$tag.err || { tail -20 gpurun_out/r06_bench_$tag.err; exit 1; }
cp gpurun_out/bench_detail_last.json gpurun_out/r06_bench_${tag}_detail.json
python3 -c "
import json; d=json.load(open('gpurun_out/r06_bench_$tag.json')); r=d['roofline']
print('value', round(d['value']/1e6,1), 'cold', round(d['cold_start_value']/1e6,1), 'ms', round(d['ms_per_step'],4), 'pcie', round(d['pcie_inclusive_value']/1e6,1))
print('iso', r['stage_ms_isolated'], 'pipe', r['stage_ms_pipelined'], 'spread', d['step_spread_ms'], 'sclk', d['sclk_mhz'])
print('flood', d['flood_config5']); print('bls', d['bls_config4']['share_verify_ms'], d['bls_config4']['verify_ms'], d['bls_config4']['certificate_fused_ms'])
print('per_req', d['per_request_path']['gpu_vs_openssl_mt'], d['per_request_path']['single_call_p50_us'], 'p50', d['p50_latency_ms_batch1k'])
"
