set -o pipefail
bash tools/gpu_bls_keys.sh && bash tools/gpu_round.sh test && bash tools/gpu_round.sh bench && bash tools/gpu_round.sh prof
