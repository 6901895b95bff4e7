# round 6: the three-stream headline loop (200 steps, 8 distinct batches) at key radix 13 in random
# key order vs radix 15 with every batch ordered by key index (the pipeline-level upper bound of a
# device key sort)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r06_sortpipe
mkdir -p $o
for round in 1 2; do
  echo "== r13 random" >> $o/pipe.txt
  timeout -k 10 300 python -u tools/timed_region_probe.py --steps 20 200 --reps 2 --streams 3 --events 0 --distinct 8 --radix 13 >> $o/pipe.txt 2>> $o/err.txt || { tail $o/err.txt; exit 1; }
  echo "== r13 sorted" >> $o/pipe.txt
  timeout -k 10 300 python -u tools/timed_region_probe.py --steps 20 200 --reps 2 --streams 3 --events 0 --distinct 8 --radix 13 --sort-keys >> $o/pipe.txt 2>> $o/err.txt || { tail $o/err.txt; exit 1; }
  echo "== r15 sorted" >> $o/pipe.txt
  timeout -k 10 300 python -u tools/timed_region_probe.py --steps 20 200 --reps 2 --streams 3 --events 0 --distinct 8 --radix 15 --sort-keys >> $o/pipe.txt 2>> $o/err.txt || { tail $o/err.txt; exit 1; }
done
cat $o/pipe.txt
