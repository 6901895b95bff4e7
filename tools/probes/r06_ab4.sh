# round 6: where the finish kernel's time goes -- default vs no root inversion (timing only,
# verdicts wrong) vs the up-tree on the chained one-statement multiply
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r06_ab4
mkdir -p $o
ed() {  # label lib
  if [ "$2" = default ]; then unset CBFT_LIB; else export CBFT_LIB=$PWD/$2; fi
  echo "== $1" >> $o/ed.txt
  timeout -k 10 240 python -u tools/ladder_probe.py --nkeys 4096 --reps 20 >> $o/ed.txt 2>> $o/err.txt || return 1
}
for round in 1 2; do
  ed default default && ed noinv build/lib_fx_noinv.so && ed upc build/lib_fx_upc.so || { tail $o/err.txt; exit 1; }
done
cat $o/ed.txt
