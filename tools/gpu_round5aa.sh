# Round-5 GPU checks, part aa: XCD-grouped attention block order -- tests, harness, in-step A/B.
set -u -o pipefail
O=gpurun_out/r5aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention" > $O/pytest_attn.log 2>&1 || { tail -30 $O/pytest_attn.log; exit 1; }
tail -2 $O/pytest_attn.log
H=build_gpu/attn_var/attn_base
for ord in 0,0,0 8,8,8 -1,-1,-1; do
  for cfg in "16 2048 32 32 128 1" "1 2048 32 8 128 1" "1 8192 32 8 128 1"; do
    echo "== order $ord cfg $cfg" >> $O/order.log
    PRA_ATTN_ORDER=$ord timeout -k 10 60 $H $cfg 20 0 >> $O/order.log 2>&1 || { tail -5 $O/order.log; exit 1; }
  done
done
grep -E "^==|pass=2" $O/order.log
A="xcd:attn.fwd_order=-1;attn.dq_order=-1;attn.dkdv_order=-1"
B="heavy:attn.fwd_order=0;attn.dq_order=0;attn.dkdv_order=0"
timeout -k 10 420 python tools/step_ab.py --arm "$A" --arm "$B" --rounds 4 --steps 5 > $O/step_ab_7b_b16_order.log 2>&1 \
  || { tail -20 $O/step_ab_7b_b16_order.log; exit 1; }
tail -3 $O/step_ab_7b_b16_order.log
timeout -k 10 300 python tools/step_ab.py --arm "$A" --arm "$B" --rounds 6 --steps 10 --model llama3-8b \
  --batch-per-gpu 1 > $O/step_ab_8b_b1_order.log 2>&1 || { tail -20 $O/step_ab_8b_b1_order.log; exit 1; }
tail -3 $O/step_ab_8b_b1_order.log
