set -o pipefail
export TMPDIR=/tmp
for cfg in "1 4 4 4" "0 4 4 4" "1 8 8 8" "1 8 8 12" "1 16 16 16"; do
  set -- $cfg
  CBFT_BLOCKING_SYNC=$1 GPU_MAX_HW_QUEUES=$2 CBFT_SMALL_STREAMS=$3 CBFT_ENGINE_INFLIGHT=$4 timeout -k 10 120 tools/host_bench 64 2000 1024 16 > gpurun_out/hb_$1_$2_$3_$4.json || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/hb_$1_$2_$3_$4.json')); print('blk $1 hwq $2 streams $3 inflight $4', {k: (d[k]['verifies_per_s'], d[k]['p50_us'], d[k]['calls_per_batch']) for k in ('verify_mt','verifysig_mt','single')})"
done
