#!/bin/bash
# attention microbench: timing, kernel trace, and PMC counters (separate rocprofv3 runs)
set -u
mkdir -p gpurun_out/attn
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 python tools/attn_bench.py ${ATTN_ARGS:-} > gpurun_out/attn/timing.log 2>&1 || exit $?
cat gpurun_out/attn/timing.log | tail -1
timeout -k 10 120 rocprofv3 -L > gpurun_out/attn/counters.txt 2>&1 || true
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/attn/trace -o t -- python3 tools/attn_bench.py ${ATTN_ARGS:-} --iters 3 > gpurun_out/attn/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC --kernel-trace --output-format csv -d gpurun_out/attn/pmc1 -o p -- python3 tools/attn_bench.py ${ATTN_ARGS:-} --iters 2 > gpurun_out/attn/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/attn/pmc2 -o p -- python3 tools/attn_bench.py ${ATTN_ARGS:-} --iters 2 > gpurun_out/attn/pmc2.log 2>&1 || exit $?
ls gpurun_out/attn/*
