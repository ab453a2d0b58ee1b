# make build | test | test-gpu | bench | prof | asan | lint   (the reference's gradle build + CI)
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

# host-side sanitizers (ASan + UBSan) over the native runtime: a self test of every GPU-free entry point
asan:
	mkdir -p build
	g++ -std=c++17 -g -O1 -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
	    -I/opt/rocm/include tony_amd/native/tony_native.cpp tony_amd/native/tests/native_selftest.cpp \
	    -ldl -lpthread -o build/native_selftest_asan
	ASAN_OPTIONS=detect_leaks=1 ./build/native_selftest_asan

# static checks: ruff (when installed) + byte-compilation of every module
lint:
	$(PY) -m compileall -q tony_amd tests tools bench.py __graft_entry__.py
	@if $(PY) -m ruff --version >/dev/null 2>&1; then $(PY) -m ruff check tony_amd tests tools bench.py; \
	 else echo "ruff not installed: skipped"; fi

.PHONY: build test test-gpu bench prof asan lint
