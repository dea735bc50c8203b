# Round-5 GPU checks, part w: effective clock per kernel in the 7B B16 step (GRBM PMC).
set -u -o pipefail
O=gpurun_out/r5w; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pmc_clock -o run -- python3 bench.py --steps 3 --warmup 2 > $O/pmc_clock.log 2>&1 || { tail -20 $O/pmc_clock.log; exit 1; }
python tools/pmc_clock.py $(find $O/pmc_clock -name 'run_results.db' | head -1) > $O/step_clock_7b_b16.txt 2>&1; head -30 $O/step_clock_7b_b16.txt
rm -rf $O/pmc_clock
