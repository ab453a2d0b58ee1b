set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_x3_gpu.py tests/test_ops_gpu.py -q -k "x3 or fp32 or avgpool or box3 or pool" > gpurun_out/x3_tests.log 2>&1 || { tail -30 gpurun_out/x3_tests.log; exit 1; }
tail -3 gpurun_out/x3_tests.log
timeout -k 10 900 python tools/ab.py --reps 2 --steps 10 --bench-args "--dtype fp32" old=TONY_X3_WGRAD_DIRECT=0,TONY_X3_WGRAD_THIN_GLDS=0 nodirect=TONY_X3_WGRAD_DIRECT=0 > gpurun_out/ab_fp32.log 2>&1 || { tail -30 gpurun_out/ab_fp32.log; exit 1; }
tail -12 gpurun_out/ab_fp32.log
