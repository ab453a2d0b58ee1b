set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 500 $PYT tests/test_x3_gpu.py -q > gpurun_out/x3_tests2.log 2>&1 || { tail -40 gpurun_out/x3_tests2.log; exit 1; }
tail -3 gpurun_out/x3_tests2.log
timeout -k 10 900 python tools/ab.py --reps 2 --steps 10 --bench-args "--dtype fp32" nojoin=TONY_INCEPTION_JOIN=0 nobranch=TONY_BRANCH_STREAMS=0 > gpurun_out/ab_fp32b.log 2>&1 || { tail -30 gpurun_out/ab_fp32b.log; exit 1; }
tail -12 gpurun_out/ab_fp32b.log
