#!/bin/bash
# Same-box A/B: the in-tree library vs every pytorch_operator_amd/_lib/exp/*.so, interleaved
# (tools/build_exp.sh builds the variants).  Per library: the in-situ step timeline
# (tools/step_timeline.py) and bench K=2000 x3, K=20 x2; REPS rounds of the whole set.
#   bash tools/gpu/ab_libs.sh OUT_DIR [REPS]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/ab}; REPS=${2:-2}; mkdir -p $O
export PYTHONUNBUFFERED=1
libs="in-tree $(ls pytorch_operator_amd/_lib/exp/*.so 2>/dev/null)"
for lib in $libs; do
  tag=$(basename $lib .so); L=$lib; [ "$lib" = in-tree ] && L=""
  PTO_HIP_LIB=$L timeout -k 10 200 python -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "fused_step or round3 or staged or stream_launch" > $O/pytest_$tag.log 2>&1 || { tail -30 $O/pytest_$tag.log; exit 1; }
  FB=""; case $tag in *fb*) FB=1;; esac
  PTO_TIMELINE_FB=$FB PTO_HIP_LIB=$L timeout -k 10 120 python tools/step_timeline.py --json $O/timeline_$tag.json > $O/timeline_$tag.txt 2>&1 || { cat $O/timeline_$tag.txt; exit 1; }
  echo "== $tag"; grep -E "period|one step" $O/timeline_$tag.txt
done
for rep in $(seq 1 $REPS); do
for lib in $libs; do
  tag=$(basename $lib .so); L=$lib; [ "$lib" = in-tree ] && L=""
  a=""; for i in 1 2 3; do a="$a $(PTO_HIP_LIB=$L timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --job-latency 0 2>>$O/err.log | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1; done
  b=""; for i in 1 2; do b="$b $(PTO_HIP_LIB=$L timeout -k 10 120 python bench.py --steps 20 --warmup 5 --job-latency 0 2>>$O/err.log | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1; done
  echo "$tag | K2000:$a | K20:$b" | tee -a $O/ab.txt
done
done
