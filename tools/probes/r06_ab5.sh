# round 6: the two-wave finish (butterfly root + wave inversion on wave 0, cofactor scans on
# wave 1, one product after the inversion) -- parity, then A/B against the one-wave tree
# (build/lib_fin1w.so) and the timing-only variant without the inversion (build/lib_fx_noinv.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r06_ab5
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_ed25519_gpu.py tests/test_pipeline_gpu.py > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
ed() {  # label lib
  if [ "$2" = default ]; then unset CBFT_LIB; else export CBFT_LIB=$PWD/$2; fi
  echo "== $1" >> $o/ed.txt
  timeout -k 10 240 python -u tools/ladder_probe.py --nkeys 4096 --reps 20 >> $o/ed.txt 2>> $o/err.txt || return 1
  [ "$1" = noinv ] && return 0
  timeout -k 10 240 python -u tools/timed_region_probe.py --steps 200 --reps 2 --streams 3 --events 0 >> $o/ed.txt 2>> $o/err.txt || return 1
}
for round in 1 2; do
  ed twowave default && ed onewave build/lib_fin1w.so && ed noinv build/lib_fx_noinv.so || { tail $o/err.txt; exit 1; }
done
cat $o/ed.txt
