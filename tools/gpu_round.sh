#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel stats.  Each GPU step has its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step=${1:-all}
if [[ $step == all || $step == test ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [[ $step == all || $step == bench ]]; then
  timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [[ $step == all || $step == prof ]]; then
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --no-cpu --latency-runs 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof.err" || { echo "rocprof failed"; tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof.err"; exit 1; }
  cd "$GRAFT_REPO_ROOT"; find gpurun_out/prof -name "*kernel_stats.csv" | head -3
fi
if [[ $step == all || $step == pmc ]]; then
  # one counter group per pass (gfx950 slot limits: 8 SQ, 4 TCC; FETCH_SIZE uses 3, WRITE_SIZE 2)
  cd /tmp
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
             "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAIT_INST_LDS" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d "$GRAFT_REPO_ROOT/gpurun_out/pmc$i" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --latency-runs 0 --no-extras > "$GRAFT_REPO_ROOT/gpurun_out/pmc$i.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/pmc$i.err" || { echo "pmc pass $i failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/pmc$i.err"; exit 1; }
  done
  cd "$GRAFT_REPO_ROOT"; find gpurun_out -name "*counter_collection.csv" | head
fi
