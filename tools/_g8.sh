set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 500 $PYT tests/test_conv_gpu.py tests/test_ops_gpu.py -q -k "strided or glds or fwd_dgrad_wgrad or accumulates or maxpool or pool" > gpurun_out/t8.log 2>&1 || { tail -40 gpurun_out/t8.log; exit 1; }
tail -3 gpurun_out/t8.log
timeout -k 10 900 python tools/ab.py --reps 3 --steps 20 nostrided=TONY_STRIDED_GLDS=0 > gpurun_out/ab_strided.log 2>&1 || { tail -30 gpurun_out/ab_strided.log; exit 1; }
tail -12 gpurun_out/ab_strided.log
