#!/bin/bash
# Four separate rocprofv3 --pmc passes over one command (gfx950 slot limits per pass: 8 SQ, 4 TCC;
# FETCH_SIZE takes 3 TCC slots and WRITE_SIZE 2, so each gets a pass of its own), each under its
# own hard time limit.  Counters only: no trace domains beside --kernel-trace.
#   bash tools/pmc_passes.sh <outdir> <python script> [args...]
# The program after rocprofv3's `--` is python3 itself (no launcher hop).
set -o pipefail
out=$1
shift
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  (cd /tmp && timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d "$out/pass$i" -o run -- python3 "$@") \
    > "$out/pass$i.out" 2> "$out/pass$i.err" || { echo "pmc pass $i failed"; tail -20 "$out/pass$i.err"; exit 1; }
done
echo "pmc passes done: $out"
