# Round-5 GPU checks, part n: fused backward at a 224-VGPR budget (room for an AdamW wave per SIMD).
set -u -o pipefail
O=gpurun_out/r5n; mkdir -p $O
run() { local f=$1; shift; echo "== $*" | tee -a $O/$f; timeout -k 10 120 "$@" >> $O/$f 2>&1; local rc=$?; tail -2 $O/$f; return $rc; }
PRA_BWD_FUSED=1 run check.log build_gpu/attn_var/attn_base 1 2048 32 32 128 1 3 1 both || exit 1
PRA_BWD_FUSED=1 run perf.log build_gpu/attn_var/attn_base 16 2048 32 32 128 1 10 0 bwd || exit 1
PRA_BWD_FUSED=1 run perf.log build_gpu/attn_var/attn_v256 16 2048 32 32 128 1 10 0 bwd || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention_bwd" > $O/pytest_attn.log 2>&1 || { tail -30 $O/pytest_attn.log; exit 1; }
tail -1 $O/pytest_attn.log
timeout -k 10 900 python tools/step_ab.py --rounds 3 --steps 4 --arm "split:attn.bwd_fused=0" --arm "fused:attn.bwd_fused=1" \
  --arm "split_noupd:attn.bwd_fused=0;noupdate" --arm "fused_noupd:attn.bwd_fused=1;noupdate" > $O/step_ab.log 2>&1 || { tail -30 $O/step_ab.log; exit 1; }
grep median $O/step_ab.log
