#!/bin/bash
# Round 5: kernel-trace timelines of the config #3 device-resident loop and the config #2 headline
# loop (rocprofv3 --kernel-trace only), printed for a steady-state window.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r05_trace
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $out/mixed -o run -- python3 $R/tools/mixed_probe.py --steps 20 --mixed-streams 2 > $out/mixed.out 2>&1 || { tail -20 $out/mixed.out; exit 1; }
tail -1 $out/mixed.out
f=$(find $out/mixed -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_timeline.py $f ed25519 --skip 200 --count 90 > $out/mixed_timeline.txt
cat $out/mixed_timeline.txt | head -90
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $out/headline -o run -- python3 $R/tools/timed_region_probe.py --steps 20 --reps 2 --events 0 > $out/headline.out 2>&1 || { tail -20 $out/headline.out; exit 1; }
cat $out/headline.out | tail -3
f=$(find $out/headline -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_timeline.py $f ed25519 --skip 30 --count 80 > $out/headline_timeline.txt
cat $out/headline_timeline.txt
