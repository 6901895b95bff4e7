# rehearsal of bench.py's N > 1 rank path on a one-GPU box: 2 ranks through torch.distributed.run,
# both on GPU 0, gloo process group (CBFT_BENCH_SHARED_GPU=1) -- the code an 8-GPU run executes,
# RCCL aside.  Rates are not a scaling measurement.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r06_rehearse2
mkdir -p $o
CBFT_BENCH_SHARED_GPU=1 timeout -k 10 800 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err \
  || { tail -40 $o/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$o/bench.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'value', round(d['value']/1e6,1), 'cold', round(d['cold_start_value']/1e6,1), 'pcie', round(d['pcie_inclusive_value']/1e6,1))
print('parity', d['parity']['all_exact'], d['parity']['blocks'].get('config2_headline'), d['parity']['blocks'].get('config5_flood'))
print('flood', d['flood_config5']); print('single', d.get('single_process_multi_gpu')); print('par', d['config']['parallelism'])
print('cpu', d['cpu_baseline']['value'] if d.get('cpu_baseline') else None); print('bls_sharded', d.get('bls_config4_sharded'))
"
