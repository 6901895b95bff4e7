#!/bin/bash
# Round 5: config #3 device-resident rate vs streams / work slots (up to 8 slots now), interleaved.
set -o pipefail
out=gpurun_out/r05_slots
mkdir -p $out
for rep in 1 2; do
  for cfg in 4:4 6:6 8:8; do
    st=${cfg%%:*}; sl=${cfg##*:}
    CBFT_WORK_SLOTS=$sl timeout -k 10 200 python -u tools/mixed_probe.py --mixed-streams $st > $out/s${st}_w${sl}_$rep.json 2> $out/s${st}_w${sl}_$rep.err \
      || { tail -5 $out/s${st}_w${sl}_$rep.err; exit 1; }
    echo "streams $st slots $sl rep $rep $(tail -1 $out/s${st}_w${sl}_$rep.json)"
  done
done
