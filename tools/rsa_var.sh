set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  CBFT_LIB=$PWD/build/var/lib$v.so timeout -k 10 120 python -u tools/rsa_quick.py 65536 65537 > gpurun_out/rsa_$v.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/rsa_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/rsa_$v.log)"
done
