cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r6_diag3; mkdir -p $O
port=29760
for f in 1 0 1 0; do
port=$((port+1))
PTO_DDP_FUSED=$f timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port tools/xgmi_check.py --backend gloo --nblk 256 --out $O/c$port > $O/c$port.log 2>&1
echo "== fused=$f rc=$?"; python -c "
import json
d=json.load(open('$O/c$port/rank0.json')); print({k:d.get(k) for k in ('max_diff_vs_rccl_path','error_after','all_ok')})"
done
