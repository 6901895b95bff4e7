#!/bin/bash
# Round 5: the wave-butterfly tree finish (4 waves per inversion) against the 64-lane LDS tree:
# parity of every finish form, then the headline at 200 and 20 steps.
set -o pipefail
out=gpurun_out/r05_wave
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_ed25519_gpu.py -x -q -k "finish or full_size or fixed or two_streams or many_streams" \
  --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
  for tb in 64 0; do
    CBFT_FINISH_TREE_BLOCK=$tb timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 \
      --no-extras --no-cpu --latency-runs 0 > $out/t${tb}_$rep.json 2> $out/t${tb}_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$out/t${tb}_$rep.json'));print('tree $tb rep $rep 200 steps', round(d['value']/1e6,1), round(d['ms_per_step'],4), d.get('step_spread_ms'), d['roofline']['stage_ms_pipelined'], d['roofline']['stage_ms_isolated'])"
    CBFT_FINISH_TREE_BLOCK=$tb timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
      --no-extras --no-cpu --latency-runs 0 > $out/t${tb}_20_$rep.json 2> $out/t${tb}_20_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$out/t${tb}_20_$rep.json'));print('tree $tb rep $rep 20 steps', round(d['value']/1e6,1), round(d['ms_per_step'],4))"
  done
done
for rep in 1 2; do
  for cfg in "2 1" "2 0" "3 0" "3 1"; do
    set -- $cfg
    CBFT_STAGE_ORDER=$2 timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --streams $1 \
      --no-extras --no-cpu --latency-runs 0 > $out/st$1_so$2_$rep.json 2> $out/st$1_so$2_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$out/st$1_so$2_$rep.json'));print('20 steps: streams $1 order $2 rep $rep', round(d['value']/1e6,1), round(d['ms_per_step'],4), d.get('sclk_mhz'))"
  done
done
