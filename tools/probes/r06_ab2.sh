# round 6 A/B on one box: finish root inversion on the VALU (build/lib_invvalu.so) vs the scalar
# unit (default); pair-ladder product interleaving (build/lib_muln2.so: (A,B) + 2 x 2 outputs,
# build/lib_muln4.so: (A,B) + 4 outputs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r06_ab2
mkdir -p $o
run() {  # label lib
  if [ "$2" = default ]; then unset CBFT_LIB; else export CBFT_LIB=$PWD/$2; fi
  echo "== $1" >> $o/iso.txt
  timeout -k 10 240 python -u tools/ladder_probe.py --nkeys 4096 --reps 20 >> $o/iso.txt 2>> $o/err.txt || return 1
  timeout -k 10 240 python -u tools/timed_region_probe.py --steps 200 --reps 2 --streams 3 --events 0 >> $o/iso.txt 2>> $o/err.txt || return 1
}
for round in 1 2; do
  run new default && run invvalu build/lib_invvalu.so && run muln2 build/lib_muln2.so && run muln4 build/lib_muln4.so || { tail $o/err.txt; exit 1; }
done
cat $o/iso.txt
