# Round-5 GPU checks, part t: 16x16x32 forward (fwd_pipe = 2) vs fwd_kernel / fwd_p_kernel in the harness.
set -u -o pipefail
O=gpurun_out/r5t; mkdir -p $O
H=build_gpu/attn_var/attn_base
run() { local f=$1; shift; echo "== $*" | tee -a $O/$f; timeout -k 10 120 "$@" >> $O/$f 2>&1; local rc=$?; tail -2 $O/$f; return $rc; }
PRA_FWD_PIPE=2 run check.log $H 1 2048 32 32 128 1 3 1 fwd || exit 1
PRA_FWD_PIPE=2 run check.log $H 2 1024 8 2 128 1 3 1 fwd || exit 1
for r in 1 2; do
  for p in 0 1 2; do PRA_FWD_PIPE=$p run perf.log $H 16 2048 32 32 128 1 20 0 fwd || exit 1; done
done
