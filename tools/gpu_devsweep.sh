# Device-resident pipeline sweep on the GPU box: tools/dev_pipe_probe.py (64K x 256 B batches over
# NSTREAMS streams) per library variant and stage order.  RUNS="label@lib@NSTREAMS@STAGE_ORDER ..."
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for r in ${RUNS:-base@concord-bft_amd/libcbft_hipcrypto.so@2@1}; do
  IFS=@ read -r label lib ns so <<< "$r"
  echo -n "$label: "
  CBFT_LIB=$lib NSTREAMS=$ns CBFT_STAGE_ORDER=$so timeout -k 10 150 python3 tools/dev_pipe_probe.py || { echo "$label failed"; exit 1; }
done
