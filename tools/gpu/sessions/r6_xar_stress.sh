#!/bin/bash
# round 6: the exchange's self-test at world 8 on one GPU, 200 steps, default vs full fences
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_xar_stress}; mkdir -p $O
export PYTHONUNBUFFERED=1 OMP_NUM_THREADS=2
[ -n "$QUEUES" ] && export GPU_MAX_HW_QUEUES=$QUEUES
for f in ${FENCES:-default full default}; do
  PTO_XAR_FENCE=$f timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) tools/dbg/xar_stress.py --steps ${STEPS:-200} \
    > $O/stress_$f.$RANDOM.log 2>&1 || { echo "stress $f failed"; exit 1; }
done
for l in $O/stress_*.log; do echo "== $l"; python3 -c "
import sys, json, re
rs = [json.loads(m) for m in re.findall(r'\{\"rank\".*?\"seconds\": [0-9.]+\}', open(sys.argv[1]).read())]
print(len(rs), 'ranks; failing ranks', [r['rank'] for r in rs if not r['ok']], 'steps', sorted({s for r in rs for s in r['failed_steps'] if s is not None})[:20], 'err', [r['error'] for r in rs], 'alloc', rs[0]['alloc_kind'] if rs else None, 's', max((r['seconds'] for r in rs), default=0))
" $l; done
