# round 6: full GPU suite + the driver's bench command on the current tree
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r06_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r06_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r06_pytest_gpu.log
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench2.json 2> gpurun_out/r06_bench2.err || { tail -20 gpurun_out/r06_bench2.err; exit 1; }
