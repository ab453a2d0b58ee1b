export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 700 python bench.py --steps 30 --warmup 6 > gpurun_out/auto.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; grep setup gpurun_out/auto.log; tail -1 gpurun_out/auto.log | cut -c1-150; grep -o '"conv_impl": {[^}]*}' gpurun_out/auto.log; exit $rc
