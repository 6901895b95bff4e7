# round 6: the pruned tree's full GPU suite, then the A/B (finish inversion VALU vs scalar unit,
# pair-ladder product interleaving) on the same box
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r06_pytest_gpu3.log 2>&1 || { tail -40 gpurun_out/r06_pytest_gpu3.log; exit 1; }
tail -2 gpurun_out/r06_pytest_gpu3.log
bash tools/probes/r06_ab2.sh
