#!/bin/bash
# round 6: the world-8 exchange stress with a ninth process holding a GPU context on the card
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r6_w8_ninth}; mkdir -p $O
export PYTHONUNBUFFERED=1 GPU_MAX_HW_QUEUES=1 OMP_NUM_THREADS=2
timeout -k 5 200 python -c "
import torch, time
x = torch.ones(1 << 28, device='cuda'); y = x * 2; torch.cuda.synchronize()
print('ninth process holds a context', flush=True); time.sleep(150)" > $O/ninth.log 2>&1 &
NINTH=$!
sleep 25
for mode in "--discriminate" ""; do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) tools/dbg/xar_stress.py --steps 40 $mode > $O/stress${mode// /}.log 2>&1
  echo "stress '$mode' rc=$?"
done
kill $NINTH 2>/dev/null; wait $NINTH 2>/dev/null
cat $O/ninth.log
for l in $O/stress*.log; do echo "== $l"; python3 -c "
import sys, json, re
rs = [json.loads(m) for m in re.findall(r'\{\"rank\".*?\"seconds\": [0-9.]+\}', open(sys.argv[1]).read())]
for r in rs: print(r['rank'], r['ok'], r['failed_steps'][:8], json.dumps(r['first'])[:300])
" $l; done
