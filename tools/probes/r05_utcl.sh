#!/bin/bash
# Round 5: address-translation counters of the pair ladder at 64 vs 4,096 keys (0.7 vs 43 GB of
# comb tables): is the 4 % steady-state cost of the big key set translation (UTCL1/UTCL2 misses)?
set -o pipefail
out=gpurun_out/r05_utcl
mkdir -p $out
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 60 rocprofv3 --list-avail) > $out/counters.txt 2> $out/counters.err || { tail -5 $out/counters.err; exit 1; }
grep -oE "\b(TCP|UTCL|TCC|GL2C|TA|TD)[A-Za-z0-9_]*(TRANSLATION|UTCL|TLB|XNACK|PTE)[A-Za-z0-9_]*" $out/counters.txt | sort -u > $out/tlb_counters.txt
cat $out/tlb_counters.txt | head -40
grp=$(grep -E "^TCP_UTCL1_TRANSLATION_(MISS|HIT)(_sum)?$|^TCP_UTCL1_PERMISSION_MISS(_sum)?$|^TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS" $out/tlb_counters.txt | grep -E "_sum$" | head -4 | tr '\n' ' ')
[ -z "$grp" ] && grp=$(grep -E "^TCP_UTCL1" $out/tlb_counters.txt | head -4 | tr '\n' ' ')
echo "pass counters: $grp"
[ -z "$grp" ] && exit 0
for nk in 64 4096; do
  (cd /tmp && timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d "$GRAFT_REPO_ROOT/$out/k$nk" -o run \
    -- python3 "$GRAFT_REPO_ROOT/tools/ed_pmc_probe.py" --mode headline --nkeys $nk) > $out/k$nk.out 2> $out/k$nk.err \
    || { echo "pmc k$nk failed"; tail -10 $out/k$nk.err; exit 1; }
  f=$(find $out/k$nk -name '*counter_collection.csv' | head -1)
  python3 - "$f" $nk <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "comb2_ladder" in r["Kernel_Name"] or "hash_kernel" in r["Kernel_Name"]:
        acc[(r["Kernel_Name"][:30], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print("nkeys", sys.argv[2], k, c, round(sum(v) / len(v)))
PY
done
