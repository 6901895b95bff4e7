#!/bin/bash
# Round 5: BLS phase stamps (build/lib_phases.so, -DCBFT_BLS_PHASES=1) and a kernel trace of
# tools/bls_probe.py on the default build.
set -o pipefail
out=gpurun_out/r05_bls_phases
mkdir -p $out
export TMPDIR=/tmp
CBFT_LIB=$PWD/build/lib_phases.so timeout -k 10 120 python -u tools/bls_phase_probe.py > $out/phases.txt 2> $out/phases.err \
  || { tail -5 $out/phases.err; exit 1; }
grep -E "phases|ok" $out/phases.txt | tail -8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 tools/bls_probe.py --reps 5 \
  > $out/probe.json 2> $out/prof.err || { tail -5 $out/prof.err; exit 1; }
f=$(find $out/prof -name '*kernel_stats.csv' | head -1)
cp "$f" $out/kernel_stats.csv
python3 - "$out/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if 'bls' in r['Name']:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us avg')
PY
