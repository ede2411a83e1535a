#!/bin/bash
# Diagnostic build of libpto_hip.so with the dK/dV pipeline's s_memtime stamps compiled in
# (-DPTO_ATTN_STAMPS) -> pytorch_operator_amd/_lib/diag/attn_stamps.so; tools/attn_pipe_stamps.py
# loads it through PTO_HIP_LIB.  The default build never contains the stamps.
set -e
cd "$(dirname "$0")/.."
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I csrc/kernels"
OBJ=build/diagobj; OUT=pytorch_operator_amd/_lib/diag
mkdir -p $OBJ $OUT
pids=()
for f in csrc/kernels/*.hip; do
  n=$(basename $f .hip); extra=""
  [ "$n" = attention ] && extra="-mllvm -amdgpu-mfma-vgpr-form=1"
  [ "$n" = attention_bwd_pipe ] && extra="-mllvm -amdgpu-mfma-vgpr-form=1 -fno-slp-vectorize -DPTO_ATTN_STAMPS"
  $HIPCC $FLAGS $extra -c $f -o $OBJ/$n.o & pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
$HIPCC --offload-arch=gfx950 -shared -fPIC -o $OUT/attn_stamps.so $OBJ/*.o
ls -la $OUT
