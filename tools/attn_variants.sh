#!/bin/bash
# Build one standalone attention harness per kernel variant (tools/attn_harness.cpp linked with
# csrc/kernels/attention.hip compiled under the variant's -D flags), on the CPU host:
#   tools/attn_variants.sh NAME="-DFLAG=1 ..." [NAME2="..."]   ->  build_gpu/attn_var/attn_<NAME>
# Run them on the GPU with tools/attn_variants_run.sh.
set -eu
cd "$(dirname "$0")/.."
OUT=build_gpu/attn_var
mkdir -p $OUT
HIPCC=${ROCM_PATH:-/opt/rocm}/bin/hipcc
FL="-O3 -std=c++17 --offload-arch=gfx950 -Icsrc -Icsrc/kernels"
AFL=${AFL-"-fno-honor-nans -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form"}
[ -f $OUT/attention_f32.o ] || $HIPCC $FL -c csrc/kernels/attention_f32.hip -o $OUT/attention_f32.o
[ -f $OUT/harness.o -a $OUT/harness.o -nt tools/attn_harness.cpp ] || $HIPCC $FL -c tools/attn_harness.cpp -o $OUT/harness.o
pids=()
for spec in "$@"; do
  name=${spec%%=*}
  defs=${spec#*=}
  ( $HIPCC $FL $AFL -DPRA_ATTN_HARNESS=1 $defs -c csrc/kernels/attention.hip -o $OUT/attention_$name.o \
      -Rpass-analysis=kernel-resource-usage 2> $OUT/attention_$name.res \
    && $HIPCC $FL $AFL -DPRA_ATTN_HARNESS=1 $defs -c csrc/kernels/attention_bwd_fused.hip -o $OUT/fused_$name.o \
      -Rpass-analysis=kernel-resource-usage 2> $OUT/fused_$name.res \
    && $HIPCC $FL $OUT/harness.o $OUT/attention_$name.o $OUT/fused_$name.o $OUT/attention_f32.o -o $OUT/attn_$name \
    && echo "built $OUT/attn_$name" ) &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
