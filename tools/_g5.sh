set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_conv_gpu.py -q -k "glds" > gpurun_out/glds_tests.log 2>&1 || { tail -30 gpurun_out/glds_tests.log; exit 1; }
tail -3 gpurun_out/glds_tests.log
timeout -k 10 900 python tools/ab.py --reps 3 --steps 20 noil=TONY_CONV_GLDS_IL=0 > gpurun_out/ab_il.log 2>&1 || { tail -30 gpurun_out/ab_il.log; exit 1; }
tail -12 gpurun_out/ab_il.log
