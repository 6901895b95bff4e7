# round 6: the wave-cooperative safegcd (scalar divsteps, lane-parallel limb updates) in the
# Ed25519 finish root and the BLS final exponentiation's Fp inversion.  Parity first (finish and
# BLS tests on the new library), then A/B against the scalar-unit form (build/lib_invscalar_*.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r06_ab3
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_ed25519_gpu.py -k "finish or golden or planted" tests/test_bls_gpu.py tests/test_relic_gpu.py > $o/pytest.log 2>&1 \
  || { tail -30 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
ed() {  # label lib
  if [ "$2" = default ]; then unset CBFT_LIB; else export CBFT_LIB=$PWD/$2; fi
  echo "== $1" >> $o/ed.txt
  timeout -k 10 240 python -u tools/ladder_probe.py --nkeys 4096 --reps 20 >> $o/ed.txt 2>> $o/err.txt || return 1
  timeout -k 10 240 python -u tools/timed_region_probe.py --steps 200 --reps 2 --streams 3 --events 0 >> $o/ed.txt 2>> $o/err.txt || return 1
}
bls() {
  if [ "$2" = default ]; then unset CBFT_LIB; else export CBFT_LIB=$PWD/$2; fi
  echo "== $1" >> $o/bls.txt
  timeout -k 10 240 python -u tools/bls_probe.py --reps 10 >> $o/bls.txt 2>> $o/err.txt || return 1
}
for round in 1; do
  ed wave default && ed scalar build/lib_invscalar_ed.so && bls wave default && bls scalar build/lib_invscalar_bls.so \
    || { tail $o/err.txt; exit 1; }
done
cat $o/ed.txt $o/bls.txt
