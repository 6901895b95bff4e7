set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ed25519_gpu.py -k "fixed_device_64k" tests/test_cpp_host.py > gpurun_out/r06_t1.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench1.json 2> gpurun_out/r06_bench1.err
