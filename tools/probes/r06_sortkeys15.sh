# round 6: key comb radix 15 (17 positions: 15 pair-ladder steps, 146 GB of tables at 4,096 keys)
# in random vs key-sorted order, beside radix 13 (16 steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r06_sortkeys15
mkdir -p $o
for round in 1 2; do
  for r in 13 15; do
    timeout -k 10 300 python -u tools/ladder_probe.py --nkeys 4096 --reps 20 --radix $r >> $o/iso.txt 2>> $o/err.txt || { tail $o/err.txt; exit 1; }
    timeout -k 10 300 python -u tools/ladder_probe.py --nkeys 4096 --reps 20 --radix $r --sort-keys >> $o/iso.txt 2>> $o/err.txt || { tail $o/err.txt; exit 1; }
  done
done
cat $o/iso.txt
