# Round-5 GPU checks, part ai: L2 hit rate of every kernel in the 7B B16 step (TCC PMC).
set -u -o pipefail
O=gpurun_out/r5ai; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/p -o p -- python3 bench.py --steps 2 --warmup 2 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python tools/pmc_summary.py $O/p > $O/l2_7b_b16.txt 2>&1 || true
grep -E "^[_a-zA-Z]|TCC_HIT|TCC_MISS" $O/l2_7b_b16.txt | head -90
rm -rf $O/p
