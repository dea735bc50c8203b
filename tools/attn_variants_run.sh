#!/bin/bash
# Run the harness executables built by tools/attn_variants.sh on the GPU box, interleaved (ABAB...)
# so clock drift hits every variant alike:  tools/attn_variants_run.sh "B S Hq Hkv D causal" name1 name2 ...
# Each run is under its own timeout; the first failure stops the script.
set -u
cd "$(dirname "$0")/.."
SHAPE=$1; shift
OUT=gpurun_out/attn_var
mkdir -p $OUT
for r in 1 2; do
  for n in "$@"; do
    echo "== $n round $r" | tee -a $OUT/run.log
    timeout -k 5 120 build_gpu/attn_var/attn_$n $SHAPE ${ITERS:-20} 0 ${MODE:-both} >> $OUT/run.log 2>&1 || { echo "FAILED $n rc=$?"; tail -5 $OUT/run.log; exit 1; }
  done
done
if [ "${CHECK:-1}" = "1" ]; then
  for n in "$@"; do
    echo "== $n check" | tee -a $OUT/run.log
    timeout -k 5 300 build_gpu/attn_var/attn_$n ${CHECK_SHAPE:-1 2048 32 32 128 1} 2 1 >> $OUT/run.log 2>&1 || { echo "CHECK FAILED $n rc=$?"; tail -5 $OUT/run.log; exit 1; }
  done
fi
grep -E '^==|pass=2|check' $OUT/run.log
