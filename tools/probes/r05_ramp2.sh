#!/bin/bash
# Round 5: the first ~200 batches of a run are slower (0.155 -> 0.125 ms per step): is it the
# pipeline settling (streams) or the hardware ramping (clocks sampled while it runs)?
set -o pipefail
out=gpurun_out/r05_ramp2
mkdir -p $out
for st in 1 3; do
  timeout -k 10 200 python -u tools/timed_region_probe.py --steps 20 --reps 1 --ramp 400 --streams $st > $out/ramp_st$st.jsonl 2> $out/ramp_st$st.err || { tail -20 $out/ramp_st$st.err; exit 1; }
  cat $out/ramp_st$st.jsonl
done
