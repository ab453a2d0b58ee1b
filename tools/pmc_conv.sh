# three counter passes over tools/pmc_conv.py (each its own rocprofv3 run, SIGKILL after 90 s), then the table
set -e
export TMPDIR=/tmp
R=$(pwd)
O=gpurun_out/pmc_conv
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d "$R/$O/a" -o run --output-format csv -- python3 "$R/tools/pmc_conv.py" --run
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU --kernel-trace -d "$R/$O/b" -o run --output-format csv -- python3 "$R/tools/pmc_conv.py" --run
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d "$R/$O/c" -o run --output-format csv -- python3 "$R/tools/pmc_conv.py" --run
python3 tools/pmc_conv.py --summarize $O > $O/summary.md
find $O -name "*trace*.csv" -delete
cat $O/summary.md
