# Round-5 GPU checks, part y: forward attention causal vs non-causal at the 7B shape and at H64/8.
set -u -o pipefail
O=gpurun_out/r5y; mkdir -p $O
H=build_gpu/attn_var/attn_base
for cfg in "16 2048 32 32 128 1" "16 2048 32 32 128 0" "16 2048 64 8 128 1" "16 2048 64 8 128 0"; do
  timeout -k 10 60 $H $cfg 20 0 fwd >> $O/fwd_causal_vs_full.log 2>&1 || { tail -5 $O/fwd_causal_vs_full.log; exit 1; }
done
cat $O/fwd_causal_vs_full.log
