cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r6_diag; mkdir -p $O
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/dbg/grad_diag.py > $O/g2.txt 2>$O/g2.err
grep rank $O/g2.txt
timeout -k 10 200 python tools/dbg/grad_diag.py > $O/g1.txt 2>$O/g1.err
grep rank $O/g1.txt
