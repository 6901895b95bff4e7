#!/bin/bash
# rocprofv3 kernel stats + SQ counters of the BLS config #4 phases (tools/bls_probe.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/blsprof
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/blsprof/trace" -o run -- python3 "$R/tools/bls_probe.py" > "$R/gpurun_out/blsprof/probe.json" 2> "$R/gpurun_out/blsprof/trace.err" || { echo trace failed; tail -20 "$R/gpurun_out/blsprof/trace.err"; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU_INT64 SQ_INSTS_SALU -d "$R/gpurun_out/blsprof/pmc1" -o run -- python3 "$R/tools/bls_probe.py" --reps 1 > /dev/null 2> "$R/gpurun_out/blsprof/pmc1.err" || { echo pmc failed; tail -20 "$R/gpurun_out/blsprof/pmc1.err"; exit 1; }
python3 "$R/tools/pmc_bls.py" "$R/gpurun_out/blsprof/pmc1/run_counter_collection.csv" > "$R/gpurun_out/blsprof/pmc_bls.json" || exit 1
cat "$R/gpurun_out/blsprof/probe.json"
find "$R/gpurun_out/blsprof" -name "*.csv" | head
