# Round-5 GPU checks, part g: fused attention backward (attention_bwd_fused.hip) in the standalone harness.
set -u -o pipefail
O=gpurun_out/r5g; mkdir -p $O
H=build_gpu/attn_var/attn_base
run() { local f=$1; shift; echo "== $*" | tee -a $O/$f; timeout -k 10 120 "$@" >> $O/$f 2>&1; local rc=$?; tail -4 $O/$f; return $rc; }
PRA_BWD_FUSED=1 run check_causal.log $H 1 2048 32 32 128 1 3 1 both || exit 1
PRA_BWD_FUSED=1 run check_full.log $H 1 1024 16 16 128 0 3 1 both || exit 1
PRA_BWD_FUSED=1 run check_gqa.log $H 2 1024 8 2 128 1 3 1 both || exit 1
PRA_BWD_FUSED=0 run perf.log $H 16 2048 32 32 128 1 10 0 bwd || exit 1
PRA_BWD_FUSED=1 run perf.log $H 16 2048 32 32 128 1 10 0 bwd || exit 1
PRA_BWD_FUSED=0 run perf.log $H 16 2048 32 32 128 1 10 0 bwd || exit 1
PRA_BWD_FUSED=1 run perf.log $H 16 2048 32 32 128 1 10 0 bwd || exit 1
