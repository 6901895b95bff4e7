# round 6 final tree: every GPU test, smoke, the driver's bench command, and the rocprof kernel
# statistics of the bench (separate run).  Outputs under gpurun_out/r06_final/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=$GRAFT_REPO_ROOT/gpurun_out/r06_final
mkdir -p $o
python3 tools/tree_hash.py > $o/csrc_tree.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1 \
  || { tail -30 $o/pytest_gpu.log; exit 1; }
tail -2 $o/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 500 python -u bench.py > $o/bench.json 2> $o/bench.err || { tail -30 $o/bench.err; exit 1; }
python3 - $o/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
bls = d.get("bls_config4", {})
print("value", d["value"], "cold", d.get("cold_start_value"), "ms", d["ms_per_step"], "pcie", d.get("pcie_inclusive_value"),
      "frac", d["roofline"]["frac"], "cpu", d["cpu_baseline"]["value"])
print("bls", {k: v for k, v in bls.items() if k.endswith("_ms")})
PY
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu --latency-runs 0 > $o/bench_under_rocprof.json 2> $o/prof.err \
  || { tail -20 $o/prof.err; exit 1; }
find $o/prof -name "*kernel_stats.csv" | head -2
