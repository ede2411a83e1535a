# segment-aligned slab reduction (in-tree) vs HEAD, and nontemporal fc1 param / momentum stores
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5_nt; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_kernels.txt 2>&1 || { tail -30 $O/pytest_kernels.txt; exit 1; }
tail -1 $O/pytest_kernels.txt
bash tools/gpu/ab_libs.sh $O 2
