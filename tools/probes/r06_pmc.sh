# round 6 final tree: the four PMC records (separate --pmc passes per workload, tools/pmc_passes.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=$GRAFT_REPO_ROOT/gpurun_out/r06_pmc
mkdir -p $o
bash tools/pmc_passes.sh $o/headline $GRAFT_REPO_ROOT/tools/ed_pmc_probe.py --mode headline &&
bash tools/pmc_passes.sh $o/small $GRAFT_REPO_ROOT/tools/ed_pmc_probe.py --mode small &&
bash tools/pmc_passes.sh $o/mixed $GRAFT_REPO_ROOT/tools/ed_pmc_probe.py --mode mixed &&
bash tools/pmc_passes.sh $o/bls $GRAFT_REPO_ROOT/tools/bls_probe.py --reps 1 || exit 1
timeout -k 10 200 python -u tools/lone_probe.py > $o/lone.txt 2>&1 || { tail $o/lone.txt; exit 1; }
tail -3 $o/lone.txt
