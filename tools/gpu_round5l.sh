# Round-5 GPU checks, part l: token-major row-constant pass of the fused backward.
set -u -o pipefail
O=gpurun_out/r5l; mkdir -p $O
H=build_gpu/attn_var/attn_base
run() { local f=$1; shift; echo "== $*" | tee -a $O/$f; timeout -k 10 120 "$@" >> $O/$f 2>&1; local rc=$?; tail -2 $O/$f; return $rc; }
PRA_BWD_FUSED=1 run check.log $H 1 2048 32 32 128 1 3 1 both || exit 1
PRA_BWD_FUSED=1 run check.log $H 2 1024 8 2 128 0 3 1 both || exit 1
PRA_BWD_FUSED=0 run perf.log $H 16 2048 32 32 128 1 10 0 bwd || exit 1
PRA_BWD_FUSED=1 run perf.log $H 16 2048 32 32 128 1 10 0 bwd || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > $O/pytest_attn.log 2>&1 || { tail -30 $O/pytest_attn.log; exit 1; }
tail -1 $O/pytest_attn.log
timeout -k 10 600 python tools/step_ab.py --rounds 3 --steps 4 --arm "split:attn.bwd_fused=0" --arm "fused:attn.bwd_fused=1" > $O/step_ab_fused_bwd.log 2>&1 || { tail -30 $O/step_ab_fused_bwd.log; exit 1; }
grep median $O/step_ab_fused_bwd.log
