# three counter passes over tools/pmc_glds.py (each its own rocprofv3 run, SIGKILL after 90 s)
set -e
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/pmc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d "$R/gpurun_out/pmc/a" -o run --output-format csv -- python3 "$R/tools/pmc_glds.py"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU --kernel-trace -d "$R/gpurun_out/pmc/b" -o run --output-format csv -- python3 "$R/tools/pmc_glds.py"
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d "$R/gpurun_out/pmc/c" -o run --output-format csv -- python3 "$R/tools/pmc_glds.py"
