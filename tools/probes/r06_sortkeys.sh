# round 6: table locality probe -- the isolated pair ladder on a batch in random key order vs the
# same batch ordered by key index, at key comb radix 13 (default), 14 and 11
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r06_sortkeys
mkdir -p $o
for round in 1 2; do
  for r in 13 14 11; do
    timeout -k 10 300 python -u tools/ladder_probe.py --nkeys 4096 --reps 20 --radix $r >> $o/iso.txt 2>> $o/err.txt || { tail $o/err.txt; exit 1; }
    timeout -k 10 300 python -u tools/ladder_probe.py --nkeys 4096 --reps 20 --radix $r --sort-keys >> $o/iso.txt 2>> $o/err.txt || { tail $o/err.txt; exit 1; }
  done
done
cat $o/iso.txt
