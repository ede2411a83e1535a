# Developer entry points (the reference's Makefile / Travis / Argo roles).
PY ?= python
GPURUN ?= /usr/local/graft/bin/gpurun

.PHONY: build test test-cpu test-gpu e2e bench latency schema verify clean

build:            ## HIP kernels (gfx950), operator binary, _opcore, C++ tests
	$(PY) -c "import __graft_entry__ as g; g.build()"

test: test-cpu    ## CPU suite (what CI runs without a GPU; tools/ci.sh cpu = build + verify + this)

test-cpu: build
	$(PY) -m pytest tests -m "not gpu" -q

test-gpu: build   ## on an MI355X (locally or through gpurun)
	$(PY) -m pytest tests -m gpu -q

e2e: build        ## operator e2e against the local cluster
	$(PY) -m pytest tests/test_e2e_local.py tests/test_sdk.py -q

bench:            ## headline benchmark (1 GPU); torchrun for N > 1
	$(PY) bench.py --steps 2000 --warmup 50

latency:          ## job create -> first step
	$(PY) benchmarks/job_latency.py --replicas 1 --backend rccl --gpus 0

schema:           ## regenerate docs/pytorchjob.schema.json from the SDK models
	$(PY) tools/gen_schema.py

verify:           ## generated files up to date (the reference's verify-codegen)
	$(PY) tools/gen_schema.py --check

clean:
	rm -rf build pytorch_operator_amd/_lib/*.so pytorch_operator_amd/_lib/pytorch-operator* \
	       pytorch_operator_amd/_lib/operator-tests* pytorch_operator_amd/_lib/*.stamp
