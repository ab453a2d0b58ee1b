set -e
export TMPDIR=/tmp
R=$(pwd)
for g in 1 0; do
  TONY_POOL_BN_GATHER=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/pg$g" -o run --output-format csv -- python3 "$R/bench.py" --model resnet50 --steps 5 --warmup 5 --mode eager > gpurun_out/pg$g.log 2>&1
  python3 tools/prof_summary.py gpurun_out/pg$g --skip 6 > gpurun_out/pg${g}_summary.md
  find gpurun_out/pg$g -name '*trace*' -delete
done
