export TMPDIR=/tmp; R=$(pwd)
timeout -k 10 900 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_br" -o run --output-format csv -- python3 "$R/bench.py" --steps 8 --warmup 6 --mode eager > gpurun_out/prof_br.log 2>&1
rc=$?; python3 tools/step_union.py gpurun_out/prof_br > gpurun_out/prof_br_union.txt; rm -rf gpurun_out/prof_br; exit $rc
