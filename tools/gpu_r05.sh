#!/bin/bash
# Round-5 GPU session steps; each GPU step has its own time limit and the first failure ends the
# session.  usage: bash tools/gpu_r05.sh step [step ...]
#   test        pytest -m gpu (one process)
#   smoke       __graft_entry__.smoke()
#   bench       python bench.py (driver defaults) -> gpurun_out/bench.json
#   prof        rocprofv3 --kernel-trace --stats over a short bench -> gpurun_out/prof/
#   pmc_head    PMC passes over the headline workload -> gpurun_out/pmc_ed25519_headline.json
#   pmc_small   PMC passes over the p50 path (batches of 1,024) -> gpurun_out/pmc_ed25519_small.json
#   pmc_mixed   PMC passes over config #3 -> gpurun_out/pmc_ed25519_mixed.json
#   pmc_bls     kernel stats + PMC passes over the BLS config #4 probe -> gpurun_out/pmc_bls.json
#   phases      phase times of the fused small-batch kernel (build/lib_edphases.so, -DCBFT_ED_PHASES=1)
#   trace       kernel trace of the device-resident two-stream pipeline (overlap of the stages)
#   ab          interleaved A/B of $LIBS (tools/ab_libs.sh)
#   blsphases   phase times of the BLS signing kernel (build/lib_blsphases.so, -DCBFT_BLS_PHASES=1)
#   reqsweep    per-request path under $VARIANTS (tools/gpu_reqsweep.sh)
#   abmix       the same over config #3 only (tools/mixed_probe.py)
#   san         host-layer ASan+UBSan / TSan runs (make sanitize first)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    test)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
      tail -3 gpurun_out/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
        || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
      cat gpurun_out/smoke.log ;;
    bench)
      timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err \
        || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
      wc -c gpurun_out/bench.json; tail -c 2500 gpurun_out/bench.json ;;
    bench20)  # the driver's command line
      timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench20.json 2> gpurun_out/bench20.err \
        || { echo "bench failed"; tail -30 gpurun_out/bench20.err; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/bench20.json'));print({k: d[k] for k in ('value', 'ms_per_step', 'step_spread_ms', 'sclk_mhz', 'comb_radix_cliff', 'pcie_inclusive_value', 'p50_latency_ms_batch1k')}); print(d['roofline']['frac'], d['roofline']['stage_ms_pipelined'], d['mixed_config3']['device_resident_value'], d['bls_config4'])" ;;
    prof)
      (cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run \
        -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu) > gpurun_out/prof_bench.json 2> gpurun_out/prof.err \
        || { echo "rocprof failed"; tail -30 gpurun_out/prof.err; exit 1; }
      find gpurun_out/prof -name "*kernel_stats.csv" | head -3 ;;
    pmc_head|pmc_small|pmc_mixed)
      mode=${step#pmc_}; [ "$mode" = head ] && mode=headline
      bash tools/pmc_passes.sh "$R/gpurun_out/pmc_$mode" "$R/tools/ed_pmc_probe.py" --mode $mode || exit 1
      python3 tools/pmc_record.py "$R/gpurun_out/pmc_$mode" "ed_pmc_probe --mode $mode" ed25519_ \
        > gpurun_out/pmc_ed25519_$mode.json || exit 1 ;;
    pmc_bls)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/blsprof/trace" -o run \
        -- python3 "$R/tools/bls_probe.py") > gpurun_out/blsprof_probe.json 2> gpurun_out/blsprof_trace.err \
        || { echo "bls trace failed"; tail -20 gpurun_out/blsprof_trace.err; exit 1; }
      cat gpurun_out/blsprof_probe.json
      bash tools/pmc_passes.sh "$R/gpurun_out/pmc_bls" "$R/tools/bls_probe.py" --reps 1 || exit 1
      python3 tools/pmc_record.py --longest "$R/gpurun_out/pmc_bls" "bls_probe --reps 1 (config #4)" bls_ \
        > gpurun_out/pmc_bls.json || exit 1 ;;
    ab)
      bash tools/ab_libs.sh || exit 1 ;;
    blsphases)
      CBFT_LIB=$R/build/lib_blsphases.so timeout -k 10 120 python3 -u tools/bls_probe.py --reps 2 > gpurun_out/bls_phases.log 2>&1 \
        || { echo "bls phase probe failed"; tail -20 gpurun_out/bls_phases.log; exit 1; }
      grep -E "sign|{" gpurun_out/bls_phases.log | tail -12 ;;
    reqsweep)
      bash tools/gpu_reqsweep.sh || exit 1 ;;
    abmix)
      MODE=mixed bash tools/ab_libs.sh || exit 1 ;;
    phases)
      CBFT_LIB=$R/build/lib_edphases.so timeout -k 10 120 python3 -u tools/ed_small_probe.py > gpurun_out/ed_phases.log 2>&1 \
        || { echo "phase probe failed"; tail -20 gpurun_out/ed_phases.log; exit 1; }
      grep -E "us|verdicts" gpurun_out/ed_phases.log | head -20 ;;
    trace)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace" -o run \
        -- python3 "$R/tools/dev_pipe_probe.py") > gpurun_out/trace_probe.log 2>&1 \
        || { echo "trace failed"; tail -20 gpurun_out/trace_probe.log; exit 1; }
      tail -2 gpurun_out/trace_probe.log
      f=$(find gpurun_out/trace -name "*kernel_trace.csv" | head -1)
      python3 tools/trace_timeline.py "$f" ed25519_ --skip 60 --count 40 ;;
    san)
      bash tools/sanitize.sh || { echo "sanitizer runs failed"; exit 1; } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
