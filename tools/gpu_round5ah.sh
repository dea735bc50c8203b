# Round-5 GPU checks, part ah: attention PMC (B16 S2048 H32 D128 causal) with the heavy-first and the
# XCD-grouped block order: issue mix, MFMA busy, L2 hit rate.
set -u -o pipefail
O=gpurun_out/r5ah; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="--B 16 --S 2048 --Hq 32 --Hkv 32 --D 128"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for mode in heavy xcd; do
  ORD=-1; [ $mode = heavy ] && ORD=0
  for pass in 1 2 3; do
    eval P=\$P$pass
    PYRECOVER_ATTN_FWD_ORDER=$ORD PYRECOVER_ATTN_DQ_ORDER=$ORD PYRECOVER_ATTN_DKDV_ORDER=$ORD timeout -k 10 120 \
      rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/${mode}_p$pass -o p -- python3 tools/attn_bench.py $A --iters 2 \
      > $O/${mode}_p$pass.log 2>&1 || { tail -20 $O/${mode}_p$pass.log; exit 1; }
  done
  python tools/pmc_summary.py $O/${mode}_p1 $O/${mode}_p2 $O/${mode}_p3 > $O/attn_pmc_${mode}.txt 2>&1 || true
  head -80 $O/attn_pmc_${mode}.txt
done
rm -rf $O/*_p1 $O/*_p2 $O/*_p3
