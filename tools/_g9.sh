set -u
set -u
timeout -k 10 300 python tools/conv_bench.py --tony > gpurun_out/conv_bench_tony2.log 2>&1 || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH_ARGS="--model resnet50" bash tools/gpu_steps.sh prof || exit $?
cp gpurun_out/prof_summary.md gpurun_out/r50_prof_summary.md; cp gpurun_out/prof_by_grid.md gpurun_out/r50_prof_by_grid.md
bash tools/gpu_steps.sh bench2_nomarkers; echo "nomarkers rc=$?"
bash tools/gpu_steps.sh ps_job || exit $?
