# round 6: the table-size cost of wider combs with the step count held: key radix 13 vs 14 (20 vs 19
# positions, both 16 pair-ladder steps), B radix 22 vs 24 (12 vs 11 positions, 16 steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r06_radix
mkdir -p $o
for round in 1 2; do
  for cfg in "13 22" "14 22" "13 24" "14 24"; do
    set -- $cfg
    echo "== key $1 B $2" >> $o/iso.txt
    timeout -k 10 300 python -u tools/ladder_probe.py --nkeys 4096 --reps 20 --radix $1 --b-radix $2 >> $o/iso.txt 2>> $o/err.txt || { tail $o/err.txt; exit 1; }
  done
done
cat $o/iso.txt
