# Round-5 GPU checks, part af: wave pairing in 8-wave causal attention blocks (PRA_ATTN_ORDER f,q,k,pair).
set -u -o pipefail
O=gpurun_out/r5af; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py \
  -k "block_order or attention_bwd_dkdv_kernels or attention_fwd" > $O/pytest_pair.log 2>&1 || { tail -30 $O/pytest_pair.log; exit 1; }
tail -2 $O/pytest_pair.log
H=build_gpu/attn_var/attn_base
PRA_ATTN_ORDER=-1,-1,-1,1 timeout -k 10 120 $H 1 2048 32 32 128 1 3 1 > $O/check_pair.log 2>&1 || { cat $O/check_pair.log; exit 1; }
grep -h check $O/check_pair.log
for rep in 1 2; do
for ord in -1,-1,-1,0 -1,-1,-1,1; do
  for cfg in "16 2048 32 32 128 1" "1 8192 32 8 128 1" "16 2048 32 8 128 1"; do
    echo "== order $ord rep $rep cfg $cfg" >> $O/pair.log
    PRA_ATTN_ORDER=$ord timeout -k 10 60 $H $cfg 20 0 >> $O/pair.log 2>&1 || { tail -5 $O/pair.log; exit 1; }
  done
done
done
grep -E "^==|pass=2" $O/pair.log
