# round-end check on the final tree: the whole GPU suite (unbuffered, as the driver runs it),
# smoke(), the driver-shaped bench (K=20 / W=5) and K=2000, and the step timeline
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5_final; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread \
  > $O/pytest_gpu_full.txt 2>&1 || { tail -40 $O/pytest_gpu_full.txt; exit 1; }
tail -2 $O/pytest_gpu_full.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_k20_$i.json 2>> $O/bench_err.txt || exit 1
done
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 > $O/bench_k2000.json 2>> $O/bench_err.txt || exit 1
grep -ho '"ms_per_step": [0-9.]*' $O/bench_k*.json
timeout -k 10 150 python tools/step_timeline.py --json $O/timeline.json > $O/timeline.txt 2>&1 || exit 1
head -3 $O/timeline.txt
