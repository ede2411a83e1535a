# slab reduction workgroups aligned to the chunk-row segment, and the fc gradient tiles on
# conv_bwd4's group B (PTO_FC_BWD4=1): kernel tests both ways, then the A/B against HEAD's library
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5_seg; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_kernels.txt 2>&1 || { tail -30 $O/pytest_kernels.txt; exit 1; }
tail -1 $O/pytest_kernels.txt
PTO_FC_BWD4=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_kernels_fcb4.txt 2>&1 || { tail -30 $O/pytest_kernels_fcb4.txt; exit 1; }
tail -1 $O/pytest_kernels_fcb4.txt
AB_ENVS="fcb4:PTO_FC_BWD4=1" TL_ARGS="--by-mod tail:610 --by-mod conv_bwd4:4" bash tools/gpu/ab_libs.sh $O 2
