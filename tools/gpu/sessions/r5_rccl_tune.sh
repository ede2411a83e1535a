# RCCL env candidates under a real RCCL communicator (one rank): the GPU test, then the full
# candidate list with the tool's defaults
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5_rccl_tune; mkdir -p $O
export PYTHONUNBUFFERED=1
PTO_TEST_RECORD_DIR=$O timeout -k 10 320 python -u -m pytest tests/test_rccl_gpu.py -x -q --timeout 300 \
  --timeout-method thread -k tune > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 600 python tools/rccl_tune.py --nproc 1 --out $O/rccl_tune_w1_all.json > $O/tune.txt 2>&1 || { tail -20 $O/tune.txt; exit 1; }
cat $O/tune.txt
