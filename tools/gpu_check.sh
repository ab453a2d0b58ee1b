#!/bin/bash
# One GPU-box session: kernel numerics tests, then short benches.
# Stops at the first GPU fault / abort / timeout (exit codes other than 0/1).
set -u
mkdir -p gpurun_out
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -5 "gpurun_out/$name.log" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    tests) step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    smoke) step smoke 600 python __graft_entry__.py smoke ;;
    bench_eager) step bench_eager 900 python bench.py --steps 10 --warmup 4 --no-graph --no-miopen-find ;;
    bench) step bench 900 python bench.py --steps 20 --warmup 6 ;;
    bench_stock) step bench_stock 900 python bench.py --steps 10 --warmup 4 --no-graph --stock ;;
    prof) export TMPDIR=/tmp; R=$(pwd)
          step prof 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 5 --no-graph --no-miopen-find ${BENCH_ARGS:-}
          python3 tools/prof_summary.py gpurun_out/prof --skip 6 > gpurun_out/prof_summary.md; find gpurun_out/prof -name '*trace*' -delete ;;
    prof_graph) export TMPDIR=/tmp; R=$(pwd)   # the headline configuration: HIP graph + MIOpen find
          step prof_graph 1100 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_graph" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 6 ${BENCH_ARGS:-}
          python3 tools/prof_summary.py gpurun_out/prof_graph --skip 8 --top 100 > gpurun_out/prof_graph_summary.md
          python3 tools/prof_summary.py gpurun_out/prof_graph --skip 8 --sequence > gpurun_out/prof_graph_sequence.txt || true
          find gpurun_out/prof_graph -name '*trace*' -delete ;;
    prof_stock) export TMPDIR=/tmp; R=$(pwd)
          step prof_stock 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_stock" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 5 --no-graph --no-miopen-find --stock
          python3 tools/prof_summary.py gpurun_out/prof_stock --skip 6 > gpurun_out/prof_stock_summary.md; find gpurun_out/prof_stock -name '*trace*' -delete ;;
    bench_serial) step bench_serial 900 python bench.py --steps 20 --warmup 6 --no-wgrad-stream ;;
    bench_imm) step bench_imm 1100 python bench.py --steps 20 --warmup 6 --no-miopen-find ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
  esac
done
