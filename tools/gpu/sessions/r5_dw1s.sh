# conv_bwd4 dW_conv1 items split by px halves over both wave groups (PTO_DW1_SPLIT): tests, A/B
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5_dw1s; mkdir -p $O
PTO_HIP_LIB=pytorch_operator_amd/_lib/exp/dw1s.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest_dw1s_all.txt 2>&1 || { tail -30 $O/pytest_dw1s_all.txt; exit 1; }
tail -1 $O/pytest_dw1s_all.txt
bash tools/gpu/ab_libs.sh $O 2
