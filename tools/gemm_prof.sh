#!/bin/bash
# PMC passes over the hand-written GEMMs vs each other (tools/gemm_pmc.py); one counter group per
# rocprofv3 run. Output: gpurun_out/gemm_pmc/<kernel>_p<N>/
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/gemm_pmc
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
P3="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY TCC_HIT_sum TCC_MISS_sum"
P4="FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY"
[ -f $O/counters.txt ] || timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
for k in ${KERNELS:-nt nt32 wgrad}; do
  timeout -s KILL 90 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $O/${k}_p1 -o p -- python3 tools/gemm_pmc.py --kernel $k ${GEMM_ARGS:-} > $O/${k}_p1.log 2>&1 || { echo "pass $k 1 failed"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d $O/${k}_p2 -o p -- python3 tools/gemm_pmc.py --kernel $k ${GEMM_ARGS:-} > $O/${k}_p2.log 2>&1 || echo "pass $k 2 failed (counter names?)"
  timeout -s KILL 90 rocprofv3 --pmc $P3 --kernel-trace --output-format csv -d $O/${k}_p3 -o p -- python3 tools/gemm_pmc.py --kernel $k ${GEMM_ARGS:-} > $O/${k}_p3.log 2>&1 || echo "pass $k 3 failed (counter names?)"
  timeout -s KILL 90 rocprofv3 --pmc $P4 --kernel-trace --output-format csv -d $O/${k}_p4 -o p -- python3 tools/gemm_pmc.py --kernel $k ${GEMM_ARGS:-} > $O/${k}_p4.log 2>&1 || echo "pass $k 4 failed (counter names?)"
done
python3 tools/pmc_summary.py $O/*_p[1234] --filter gemm > $O/summary.txt 2>&1 || true
python3 tools/pmc_summary.py $O/*_p[1234] --filter wgrad >> $O/summary.txt 2>&1 || true
python3 tools/pmc_summary.py $O/*_p[1234] --filter Cijk >> $O/summary.txt 2>&1 || true
