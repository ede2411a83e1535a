#!/bin/bash
# Variant / diagnostic builds of libpto_hip.so that differ only in attention_bwd_pipe.hip's
# defines, for same-box A/B through PTO_HIP_LIB:
#   tools/build_diag_attn.sh                       -> _lib/diag/attn_stamps.so (-DPTO_ATTN_STAMPS:
#                                                     the dK/dV pipeline's s_memtime stamps,
#                                                     read by tools/attn_pipe_stamps.py)
#   tools/build_diag_attn.sh NAME "DEFS" [...]     -> _lib/diag/NAME.so per pair (the round-4
#                                                     ablation knobs were removed in round 5)
# The default build never contains the stamps.
set -e
cd "$(dirname "$0")/.."
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I csrc/kernels"
OBJ=build/diagobj; OUT=pytorch_operator_amd/_lib/diag
mkdir -p $OBJ $OUT
[ $# -eq 0 ] && set -- attn_stamps "-DPTO_ATTN_STAMPS"
pids=()
for f in csrc/kernels/*.hip; do
  n=$(basename $f .hip); [ "$n" = attention_bwd_pipe ] && continue
  extra=""; [ "$n" = attention ] && extra="-mllvm -amdgpu-mfma-vgpr-form=1"
  [ $OBJ/$n.o -nt $f ] && [ $OBJ/$n.o -nt csrc/kernels/attention_common.h ] || { $HIPCC $FLAGS $extra -c $f -o $OBJ/$n.o & pids+=($!); }
done
names=()
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  $HIPCC $FLAGS -mllvm -amdgpu-mfma-vgpr-form=1 -fno-slp-vectorize $defs -c csrc/kernels/attention_bwd_pipe.hip -o $OBJ/pipe_$name.o & pids+=($!)
  names+=($name)
done
for p in "${pids[@]}"; do wait $p; done
others=$(ls $OBJ/*.o | grep -v "/pipe_")
for name in "${names[@]}"; do
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o $OUT/$name.so $OBJ/pipe_$name.o $others
done
ls -la $OUT
