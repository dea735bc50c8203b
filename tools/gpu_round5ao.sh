# Round-5 GPU checks, part ao: SwiGLU-backward epilogue depth (row blocks of g / u in flight).
set -u -o pipefail
O=gpurun_out/r5ao; mkdir -p $O
for rep in 1 2; do
for d in 3 4 5 6; do
  timeout -k 10 120 build_gpu/nt_d$d 32768 11008 4096 2 2 > $O/nt_epi2_d${d}_r$rep.log 2>&1 || { cat $O/nt_epi2_d${d}_r$rep.log; exit 1; }
  echo "depth $d rep $rep: $(cat $O/nt_epi2_d${d}_r$rep.log)"
done
done
timeout -k 10 120 build_gpu/nt_d3 32768 11008 4096 2 0 > $O/nt_epi0.log 2>&1 || { cat $O/nt_epi0.log; exit 1; }
echo "plain: $(cat $O/nt_epi0.log)"
