# conv_bwd4: group B computes 8 of the 32 dcol tiles (2a) before its 2b (PTO_2A_SPLIT) -- A/B
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5_split; mkdir -p $O
PTO_HIP_LIB=pytorch_operator_amd/_lib/exp/split.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest_split_all.txt 2>&1 || { tail -30 $O/pytest_split_all.txt; exit 1; }
tail -1 $O/pytest_split_all.txt
TL_ARGS="--by-mod conv_bwd4:4" bash tools/gpu/ab_libs.sh $O 2
