#!/bin/bash
# A/B of library variants on the GPU box, interleaved (A B A B ...) to see through box noise.
#   LIBS="label=path[@ENV=V,ENV=V] label=path ..." ROUNDS=2 bash tools/ab_libs.sh   (path "default" = the
#   in-tree library; the optional @ part sets environment variables for that variant)
# Per variant and round: tools/ladder_probe.py (isolated stage times, verdicts checked) and a
# 100-step bench.py without extras (headline + device-resident value), each under its own limit.
# MODE=mixed: tools/mixed_probe.py only (config #3 device-resident rate and hash stage).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for r in $(seq 1 "${ROUNDS:-2}"); do
  for lv in $LIBS; do
    label=${lv%%=*}; spec=${lv#*=}; lib=${spec%%@*}; envs=""
    [[ $spec == *@* ]] && envs=$(echo "${spec#*@}" | tr ',' ' ')
    [ "$lib" = default ] && lib=$PWD/concord-bft_amd/libcbft_hipcrypto.so
    if [ "${MODE:-}" = mixed ]; then  # config #3 device-resident rate + hash stage only
      env $envs CBFT_LIB=$lib timeout -k 10 200 python -u tools/mixed_probe.py > gpurun_out/ab/mixed_${label}_$r.json 2> gpurun_out/ab/mixed_${label}_$r.err \
        || { echo "mixed $label failed"; tail -5 gpurun_out/ab/mixed_${label}_$r.err; exit 1; }
      echo "$label r$r mixed: $(tail -1 gpurun_out/ab/mixed_${label}_$r.json)"
      continue
    fi
    env $envs CBFT_LIB=$lib timeout -k 10 200 python -u tools/ladder_probe.py --reps 20 ${PROBE_ARGS:-} > gpurun_out/ab/probe_${label}_$r.json 2> gpurun_out/ab/probe_${label}_$r.err \
      || { echo "probe $label failed"; tail -5 gpurun_out/ab/probe_${label}_$r.err; exit 1; }
    env $envs CBFT_LIB=$lib timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-extras --no-cpu --latency-runs 100 ${BENCH_ARGS:-} > gpurun_out/ab/bench_${label}_$r.json 2> gpurun_out/ab/bench_${label}_$r.err \
      || { echo "bench $label failed"; tail -5 gpurun_out/ab/bench_${label}_$r.err; exit 1; }
    python3 - "$label" "$r" <<'PY'
import json, sys
label, r = sys.argv[1], sys.argv[2]
p = json.loads(open(f"gpurun_out/ab/probe_{label}_{r}.json").read().strip().splitlines()[-1])
b = json.loads(open(f"gpurun_out/ab/bench_{label}_{r}.json").read().strip().splitlines()[-1])
print(f"{label} r{r}: iso us {p['us']} ok={p['verdicts_ok']} | value (HBM-resident) {b['value']/1e6:.1f} M/s "
      f"pcie-incl {b['pcie_inclusive_value']/1e6:.1f} M/s ladder_pipe {b['roofline']['kernel_ms']*1e3:.1f} us "
      f"frac {b['roofline']['frac']:.3f} p50@1K {b.get('p50_latency_ms_batch1k') or 0:.4f} ms", flush=True)
PY
  done
done
