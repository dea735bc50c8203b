# Round-5 GPU checks, part z: XCD-grouped block order of the attention grids (PRA_ATTN_ORDER f,q,k).
set -u -o pipefail
O=gpurun_out/r5z; mkdir -p $O
H=build_gpu/attn_var/attn_base
PRA_ATTN_ORDER=2,2,2 timeout -k 10 120 $H 1 2048 32 32 128 1 3 1 > $O/check_g2.log 2>&1 || { cat $O/check_g2.log; exit 1; }
PRA_ATTN_ORDER=-1,-1,-1 timeout -k 10 120 $H 1 2048 32 8 128 1 3 1 > $O/check_auto_gqa.log 2>&1 || { cat $O/check_auto_gqa.log; exit 1; }
grep -h check $O/check_*.log
for rep in 1 2; do
for ord in 0,0,0 1,1,1 2,2,2 4,4,4 -1,-1,-1; do
  for cfg in "16 2048 32 32 128 1" "1 8192 32 8 128 1" "16 2048 32 8 128 1"; do
    echo "== order $ord rep $rep cfg $cfg" >> $O/order.log
    PRA_ATTN_ORDER=$ord timeout -k 10 60 $H $cfg 20 0 >> $O/order.log 2>&1 || { tail -5 $O/order.log; exit 1; }
  done
done
done
grep -E "^==|pass=2" $O/order.log
