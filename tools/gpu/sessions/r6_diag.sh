cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r6_diag; mkdir -p $O
export PTO_XGMI_ANY_BACKEND=1
for s in 6 12; do
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2953$s tools/ddp_parity.py --steps $s > $O/p$s.txt 2>$O/p$s.err
python -c "
import json; d=json.loads([l for l in open('$O/p$s.txt').read().strip().splitlines() if l.startswith('{')][-1])
print($s, json.dumps(d['rccl']), json.dumps(d['xgmi']))
"
done
timeout -k 10 300 python -u -m pytest tests/test_torch_parity_gpu.py -v --timeout 300 --timeout-method thread > $O/pt.log 2>&1; grep -E "PASS|FAIL|^E " $O/pt.log | head
