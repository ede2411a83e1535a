# after bench.py's kernel-argument pin: the bench GPU tests, smoke() and the driver-shaped bench
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5_final2; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_bench_gpu.py tests/test_rccl_gpu.py -q -m gpu --timeout 300 \
  --timeout-method thread > $O/pytest_bench_rccl.txt 2>&1 || { tail -40 $O/pytest_bench_rccl.txt; exit 1; }
tail -1 $O/pytest_bench_rccl.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_k20_$i.json 2>> $O/bench_err.txt || exit 1
done
grep -ho '"ms_per_step": [0-9.]*' $O/bench_k20_*.json
