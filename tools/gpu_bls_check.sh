set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bls_gpu.py tests/test_relic_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_bls.log 2>&1 || { tail -30 gpurun_out/pytest_bls.log; exit 1; }
tail -3 gpurun_out/pytest_bls.log
timeout -k 10 120 python -u tools/bls_probe.py > gpurun_out/bls_probe.json 2>&1 || { tail -20 gpurun_out/bls_probe.json; exit 1; }
cat gpurun_out/bls_probe.json
CBFT_BLS_KEYS=lane timeout -k 10 120 python -u tools/bls_probe.py --reps 1 > gpurun_out/bls_probe_lane.json 2>&1 || { tail -20 gpurun_out/bls_probe_lane.json; exit 1; }
cat gpurun_out/bls_probe_lane.json
CBFT_LIB=$PWD/concord-bft_amd/libcbft_phases.so timeout -k 10 200 python -u tools/bls_phase_probe.py > gpurun_out/phases.log 2>&1; tail -12 gpurun_out/phases.log
