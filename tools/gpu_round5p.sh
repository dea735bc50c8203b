# Round-5 GPU checks, part p: attention PMC at HEAD (B16 S2048 H32 D128 causal): split and fused backward.
set -u -o pipefail
O=gpurun_out/r5p; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="--B 16 --S 2048 --Hq 32 --Hkv 32 --D 128"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for mode in split fused; do
  F=0; [ $mode = fused ] && F=1
  PYRECOVER_ATTN_BWD_FUSED=$F timeout -k 10 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $O/${mode}_p1 -o p -- python3 tools/attn_bench.py $A --iters 2 > $O/${mode}_p1.log 2>&1 || { tail -20 $O/${mode}_p1.log; exit 1; }
  PYRECOVER_ATTN_BWD_FUSED=$F timeout -k 10 120 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d $O/${mode}_p2 -o p -- python3 tools/attn_bench.py $A --iters 2 > $O/${mode}_p2.log 2>&1 || { tail -20 $O/${mode}_p2.log; exit 1; }
  python tools/pmc_summary.py $O/${mode}_p1 $O/${mode}_p2 > $O/attn_pmc_${mode}.txt 2>&1 || true
  head -60 $O/attn_pmc_${mode}.txt
done
rm -rf $O/*_p1 $O/*_p2
