# Round-5 GPU checks, part an: per-phase stamps of the NT GEMM at the 7B W2 data-gradient shape,
# plain epilogue vs the fused SwiGLU backward (EPI 2).
set -u -o pipefail
O=gpurun_out/r5an; mkdir -p $O
for e in 0 2; do
  timeout -k 10 120 build_gpu/nt 32768 11008 4096 2 $e > $O/nt_plain_epi$e.log 2>&1 || { cat $O/nt_plain_epi$e.log; exit 1; }
  timeout -k 10 120 build_gpu/nt_stamps 32768 11008 4096 2 $e > $O/nt_stamps_epi$e.log 2>&1 || { cat $O/nt_stamps_epi$e.log; exit 1; }
  echo "== epi $e"; cat $O/nt_plain_epi$e.log $O/nt_stamps_epi$e.log
done
