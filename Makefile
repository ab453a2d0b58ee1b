# make build | test | test-gpu | bench | prof   (the reference's gradle build + CI)
PY ?= python3

build:
	$(PY) -c "import __graft_entry__ as g; g.build()"

test:
	$(PY) -m pytest tests -x -q -m "not gpu"

test-gpu: build
	$(PY) -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread

bench: build
	$(PY) bench.py --steps 20 --warmup 6

prof: build
	bash tools/gpu_check.sh prof_graph

.PHONY: build test test-gpu bench prof
