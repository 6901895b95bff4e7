set -o pipefail
export TMPDIR=/tmp
for rep in 1 2; do for f in 4 6 8; do
  CBFT_ENGINE_INFLIGHT=$f timeout -k 10 120 tools/host_bench 64 2000 1024 16 > gpurun_out/hb3_f${f}_$rep.json || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/hb3_f${f}_$rep.json')); print('inflight $f rep $rep', {k: (d[k]['verifies_per_s'], d[k]['p50_us'], d[k]['calls_per_batch']) for k in ('verify_mt','verifysig_mt','single')})"
done; done
