#!/bin/bash
# Per-request path: rate and host CPU use (cores busy, CPU us per call) at several caller counts.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "nproc $(nproc), cgroup cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
for t in 64 32 128 16; do
  timeout -k 10 200 tools/host_bench $t 2000 1024 16 > gpurun_out/reqcpu_$t.json || { echo "host_bench $t failed"; exit 1; }
  python3 - "$t" <<'PY'
import json, sys
t = sys.argv[1]
d = json.load(open(f"gpurun_out/reqcpu_{t}.json"))
for leg in ("verify_mt", "single", "openssl_mt"):
    x = d[leg]
    print(f"T={t} {leg}: {x['verifies_per_s']/1e3:.1f} K/s p50 {x['p50_us']} us calls/batch {x['calls_per_batch']} "
          f"cores_busy {x['cores_busy']} cpu_us/call {x['cpu_us_per_call']}", flush=True)
PY
done
