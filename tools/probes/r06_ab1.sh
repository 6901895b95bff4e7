# round 6 A/B on one box: round-5 library vs the current tree (tree finish with the scalar-unit
# root inversion) vs the interleaved-product ladders (build/lib_muln{2,3}.so); ladder_probe =
# one batch at a time (isolated stage times), timed_region_probe = the headline loop at 200 steps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r06_ab1
mkdir -p $o
run() {  # label lib
  if [ "$2" = default ]; then unset CBFT_LIB; else export CBFT_LIB=$PWD/$2; fi
  echo "== $1" >> $o/iso.txt
  timeout -k 10 240 python -u tools/ladder_probe.py --nkeys 4096 --reps 20 >> $o/iso.txt 2>> $o/err.txt || return 1
  timeout -k 10 240 python -u tools/timed_region_probe.py --steps 200 --reps 2 --streams 3 --events 0 >> $o/iso.txt 2>> $o/err.txt || return 1
}
for round in 1 2; do
  run new default && run r05 build/lib_r05.so && run muln2 build/lib_muln2.so && run muln3 build/lib_muln3.so || { tail $o/err.txt; exit 1; }
done
unset CBFT_LIB
cat $o/iso.txt
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$o/kt -o run -- python3 $GRAFT_REPO_ROOT/tools/ladder_probe.py --nkeys 512 --reps 10) > $o/kt.out 2>&1 || { tail -20 $o/kt.out; exit 1; }
(cd /tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVES -d $GRAFT_REPO_ROOT/$o/pmc -o run -- python3 $GRAFT_REPO_ROOT/tools/ladder_probe.py --nkeys 512 --reps 5) > $o/pmc.out 2>&1 || { tail -20 $o/pmc.out; exit 1; }
echo done
