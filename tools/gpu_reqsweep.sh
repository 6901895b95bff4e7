# Per-request path sweep on the GPU box: tools/host_bench (64 threads x 2000 single verify()
# calls) under engine / context knobs, one summary line each.  VARIANTS="label@ENV=V,ENV=V ..."
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/reqsweep
for rep in $(seq 1 "${ROUNDS:-1}"); do
  for v in ${VARIANTS:-base@X=0}; do
    label=${v%%@*}; envs=$(echo "${v#*@}" | tr ',' ' ')
    out=gpurun_out/reqsweep/${label}_$rep.json
    env $envs timeout -k 10 120 tools/host_bench ${THREADS:-64} 2000 1024 16 > $out || { echo "host_bench $label failed"; exit 1; }
    python3 -c "
import json; d=json.load(open('$out')); print('$label r$rep', {k: (round(d[k]['verifies_per_s']), d[k]['p50_us'], d[k].get('calls_per_batch')) for k in ('verify_mt','single')})"
  done
done
