#!/bin/bash
# PMC counters for the CNN-B1 layer kernels (kernel-trace only, no sys/runtime tracing).
set -o pipefail
mkdir -p gpurun_out
R=$PWD
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS \
  --output-format csv -d $R/gpurun_out/pmcA -o run -- python $R/tools/cnn_layer_bench.py --iters 3 > $R/gpurun_out/pmcA.log 2>&1 || { tail -20 $R/gpurun_out/pmcA.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum \
  --output-format csv -d $R/gpurun_out/pmcB -o run -- python $R/tools/cnn_layer_bench.py --iters 3 > $R/gpurun_out/pmcB.log 2>&1 || { tail -20 $R/gpurun_out/pmcB.log; exit 1; }
ls -R $R/gpurun_out/pmcA | head
