#!/bin/bash
# Same-box A/B of MNIST step variants, interleaved: the in-tree library, every
# pytorch_operator_amd/_lib/exp/*.so (tools/build_exp.sh builds them), and every environment
# variant named in AB_ENVS ("tag:VAR=VAL[,VAR=VAL]" entries, space-separated; run on the
# in-tree library).  Per variant: the kernel tests, the in-situ step timeline
# (tools/step_timeline.py), then REPS rounds of bench K=2000 x3 and K=20 x2.
#   AB_ENVS="tag:VAR=VAL" TL_ARGS="--by-mod conv_bwd4:4" bash tools/gpu/ab_libs.sh OUT_DIR [REPS]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/ab}; REPS=${2:-2}; mkdir -p $O
export PYTHONUNBUFFERED=1
variants="in-tree|"
for l in $(ls pytorch_operator_amd/_lib/exp/*.so 2>/dev/null); do variants="$variants $(basename $l .so)|$l"; done
for e in $AB_ENVS; do variants="$variants ${e%%:*}||${e#*:}"; done

run() {  # run <lib> <env assignments> <command...>
  local L=$1 E=$2; shift 2
  env PTO_HIP_LIB=$L ${E//,/ } "$@"
}
for v in $variants; do
  IFS='|' read -r tag L E <<< "$v"
  run "$L" "$E" timeout -k 10 200 python -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "fused or round3 or staged or stream_launch" > $O/pytest_$tag.log 2>&1 || { tail -30 $O/pytest_$tag.log; exit 1; }
  run "$L" "$E" timeout -k 10 120 python tools/step_timeline.py $TL_ARGS --json $O/timeline_$tag.json > $O/timeline_$tag.txt 2>&1 || { cat $O/timeline_$tag.txt; exit 1; }
  echo "== $tag"; grep -E "period|one step" $O/timeline_$tag.txt
done
for rep in $(seq 1 $REPS); do
for v in $variants; do
  IFS='|' read -r tag L E <<< "$v"
  a=""; for i in 1 2 3; do a="$a $(run "$L" "$E" timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --job-latency 0 2>>$O/err.log | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1; done
  b=""; for i in 1 2; do b="$b $(run "$L" "$E" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --job-latency 0 2>>$O/err.log | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1; done
  echo "$tag | K2000:$a | K20:$b" | tee -a $O/ab.txt
done
done
