# Round-5 GPU checks, part v: 4-wave 16x16x32 forward (fwd_pipe = 3) vs the others.
set -u -o pipefail
O=gpurun_out/r5v; mkdir -p $O
H=build_gpu/attn_var/attn_base
run() { local f=$1; shift; echo "== $*" | tee -a $O/$f; timeout -k 10 120 "$@" >> $O/$f 2>&1; local rc=$?; tail -2 $O/$f; return $rc; }
PRA_FWD_PIPE=3 run check.log $H 1 2048 32 32 128 1 3 1 fwd || exit 1
PRA_FWD_PIPE=3 run check.log $H 2 1024 8 2 128 1 3 1 fwd || exit 1
for r in 1 2; do
  for p in 1 2 3; do PRA_FWD_PIPE=$p run perf.log $H 16 2048 32 32 128 1 20 0 fwd || exit 1; done
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention_fwd" > $O/pytest_fwd.log 2>&1 || { tail -30 $O/pytest_fwd.log; exit 1; }
tail -1 $O/pytest_fwd.log
