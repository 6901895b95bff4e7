#!/bin/bash
# Round 5: BLS Miller lines read one line ahead (CBFT_P36_PREFETCH): BLS + RELIC GPU tests on the
# default build, then tools/bls_probe.py interleaved default / no-prefetch (build/lib_nopf.so),
# then the host-layer sanitizer runs (tools/sanitize.sh) on the same tree.
set -o pipefail
out=gpurun_out/${OUT:-r05_bls_pf}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_bls_gpu.py tests/test_relic_gpu.py -x -q --timeout 120 \
  --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2 3; do
  for v in ${VARIANTS:-default nopf}; do
    lib=$PWD/concord-bft_amd/libcbft_hipcrypto.so
    [ $v = default ] || lib=$PWD/build/lib_$v.so
    CBFT_LIB=$lib timeout -k 10 120 python -u tools/bls_probe.py --reps 10 > $out/${v}_$rep.json 2> $out/${v}_$rep.err \
      || { tail -5 $out/${v}_$rep.err; exit 1; }
    echo "$v $rep $(tail -1 $out/${v}_$rep.json)"
  done
done
[ "${SAN:-1}" = 1 ] && bash tools/sanitize.sh
exit 0
