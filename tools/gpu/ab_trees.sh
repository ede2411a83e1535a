#!/bin/bash
# Same-box A/B of whole trees, interleaved: the in-tree step against every abtree/<name>/ (a
# `git archive` of an earlier commit with its own built library; for changes that alter the
# library's C ABI, where tools/gpu/ab_libs.sh's PTO_HIP_LIB swap cannot be used).  Per tree: the
# in-situ step timeline, then REPS rounds of bench K=2000 x3 and K=20 x2.
#   bash tools/gpu/ab_trees.sh OUT_DIR [REPS]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/abt}; REPS=${2:-2}; mkdir -p $O
export PYTHONUNBUFFERED=1
trees="in-tree|."
for d in abtree/*/; do [ -f "$d/bench.py" ] && trees="$trees $(basename $d)|$d"; done
for v in $trees; do
  IFS='|' read -r tag D <<< "$v"
  (cd $D && timeout -k 10 120 python tools/step_timeline.py $TL_ARGS > $GRAFT_REPO_ROOT/$O/timeline_$tag.txt 2>&1) || { cat $O/timeline_$tag.txt; exit 1; }
  echo "== $tag"; grep -E "period|one step|phase times" $O/timeline_$tag.txt
done
for rep in $(seq 1 $REPS); do
for v in $trees; do
  IFS='|' read -r tag D <<< "$v"
  a=""; for i in 1 2 3; do a="$a $(cd $D && timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --job-latency 0 2>>$GRAFT_REPO_ROOT/$O/err.log | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1; done
  b=""; for i in 1 2; do b="$b $(cd $D && timeout -k 10 120 python bench.py --steps 20 --warmup 5 --job-latency 0 2>>$GRAFT_REPO_ROOT/$O/err.log | grep -o '"ms_per_step": [0-9.]*' | cut -d' ' -f2)" || exit 1; done
  echo "$tag | K2000:$a | K20:$b" | tee -a $O/ab.txt
done
done
