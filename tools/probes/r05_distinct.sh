#!/bin/bash
# Round 5: is the late-run speed-up cache reuse of the repeated batch?  The ramp with 1 batch
# repeated vs 8 distinct batches cycled (same 4,096 keys, different messages: different digits).
set -o pipefail
out=gpurun_out/r05_distinct
mkdir -p $out
for d in 1 8; do
  timeout -k 10 300 python -u tools/timed_region_probe.py --steps 20 200 --reps 2 --ramp 400 --streams 3 --distinct $d \
    > $out/d$d.jsonl 2> $out/d$d.err || { tail -20 $out/d$d.err; exit 1; }
  python3 -c "
import json
for l in open('$out/d$d.jsonl'):
    r = json.loads(l); r.pop('clock_samples_ms_mhz', None); print('distinct $d', r)"
done
