#!/bin/bash
# Round 5: instruction-fetch counters of the pair ladder (headline batches): is the ladder's
# two-waves-per-SIMD overlap bounded by instruction fetch?
set -o pipefail
out=gpurun_out/r05_ifetch
mkdir -p $out
export TMPDIR=/tmp
i=0
for grp in "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_BUSY_CYCLES SQC_ICACHE_REQ"; do
  i=$((i + 1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d "$GRAFT_REPO_ROOT/$out/pass$i" -o run \
    -- python3 "$GRAFT_REPO_ROOT/tools/ed_pmc_probe.py" --mode headline) > $out/pass$i.out 2> $out/pass$i.err \
    || { echo "pass $i failed"; tail -5 $out/pass$i.err; exit 1; }
  f=$(find $out/pass$i -name '*counter_collection.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    if "comb2_ladder" in k or "hash_kernel" in k or "finish_tree" in k:
        acc[(k[:28], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(k, c, round(sum(v) / len(v)))
PY
done
