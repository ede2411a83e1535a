#!/bin/bash
# Build -D experiment variants of libpto_hip.so for same-box A/B (tools/gpu/ab_libs.sh loads
# every pytorch_operator_amd/_lib/exp/*.so through PTO_HIP_LIB).  Every experiment library also
# links csrc/kernels/experiments/*.hip (the rejected attention variants; `tools/build_exp.sh ref ""`
# builds one with the default MNIST kernels).
#   tools/build_exp.sh name1 "-DFOO=0" name2 "-DFOO=0 -DBAR=1" ...
set -e
cd "$(dirname "$0")/.."
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I csrc/kernels"
OBJ=build/expobj; OUT=pytorch_operator_amd/_lib/exp
mkdir -p $OBJ $OUT
rm -f $OUT/*.so
pids=()
# every default source, plus csrc/kernels/experiments/*.hip: the rejected variants kept for A/B
# (attention_variants.hip: attention.hip's dispatcher reaches them through weak symbols)
for f in csrc/kernels/*.hip csrc/kernels/experiments/*.hip; do
  n=$(basename $f .hip); [ "$n" = mnist_kernels ] && continue
  extra=""; [ "$n" = attention ] && extra="${ATTN_FLAGS--mllvm -amdgpu-mfma-vgpr-form=1}"  # as ops/_native.py
  [ "$n" = attention_variants ] && extra="-mllvm -amdgpu-mfma-vgpr-form=1"
  [ "$n" = attention_bwd_pipe ] && extra="-mllvm -amdgpu-mfma-vgpr-form=1 -fno-slp-vectorize"
  [ $OBJ/$n.o -nt $f ] && [ $OBJ/$n.o -nt csrc/kernels/attention_common.h ] || { $HIPCC $FLAGS $extra -c $f -o $OBJ/$n.o & pids+=($!); }
done
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  ( $HIPCC $FLAGS $defs -c csrc/kernels/mnist_kernels.hip -o $OBJ/mnist_$name.o ) & pids+=($!)
  names+=($name)
done
for p in "${pids[@]}"; do wait $p; done
others=$(ls $OBJ/*.o | grep -v "/mnist_")
for name in "${names[@]}"; do
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o $OUT/$name.so $OBJ/mnist_$name.o $others
done
ls -la $OUT
