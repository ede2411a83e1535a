set -o pipefail
O=gpurun_out/r6_reset; mkdir -p $O
export PYTHONUNBUFFERED=1 PTO_TEST_RECORD_DIR=$O/rec
timeout -k 10 700 python -u -m pytest tests/test_bench_gpu.py tests/test_xgmi_gpu.py -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
GPU_MAX_HW_QUEUES=1 PTO_XGMI_ANY_BACKEND=1 timeout -k 10 300 python bench.py --gpus 8 --backend gloo --steps 20 --warmup 5 --job-latency 0 --json-out $O/w8_q1.json > $O/w8_q1.log 2>&1 || { tail -20 $O/w8_q1.log; exit 1; }
echo w8 done
