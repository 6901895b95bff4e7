# round 6, last tree: every GPU test, smoke and the driver's bench command (N = 1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=$GRAFT_REPO_ROOT/gpurun_out/r06_last
mkdir -p $o
python3 tools/tree_hash.py > $o/csrc_tree.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1 \
  || { tail -30 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
bash tools/probes/r06_bench.sh last
