# MFMA-utilisation counters (one pass each) for 12x128 and 12x256, plus HBM fetch bytes for 12x128
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $R/gpurun_out/pmc4_128 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-graph > $R/gpurun_out/pmc4_128.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $R/gpurun_out/pmc4_256 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-graph --channels 256 > $R/gpurun_out/pmc4_256.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc4_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-graph > $R/gpurun_out/pmc4_fetch.log 2>&1
