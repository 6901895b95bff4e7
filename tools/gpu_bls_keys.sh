set -o pipefail
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_bls_gpu.py tests/test_relic_gpu.py -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_blsk.log 2>&1 || { tail -30 gpurun_out/pytest_blsk.log; exit 1; }
tail -1 gpurun_out/pytest_blsk.log
timeout -k 10 200 python3 -u tools/bls_probe.py --reps 5 > gpurun_out/blsk_probe.json 2> gpurun_out/blsk_probe.err || { tail -5 gpurun_out/blsk_probe.err; exit 1; }
cat gpurun_out/blsk_probe.json | head -c 1500
