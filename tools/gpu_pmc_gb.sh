#!/bin/bash
# PMC counters over a short 1B-row groupBy bench (kernel-trace only; <= 8 SQ / 4 TCC per pass).
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R && mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc_gbA -o run -- python bench.py --workload groupby --steps 1 --warmup 1 > gpurun_out/pmc_gbA.log 2>&1 || { tail -20 gpurun_out/pmc_gbA.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LEVEL_WAVES SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_gbB -o run -- python bench.py --workload groupby --steps 1 --warmup 1 > gpurun_out/pmc_gbB.log 2>&1 || { tail -20 gpurun_out/pmc_gbB.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE WRITE_SIZE --output-format csv -d gpurun_out/pmc_gbC -o run -- python bench.py --workload groupby --steps 1 --warmup 1 > gpurun_out/pmc_gbC.log 2>&1 || { tail -20 gpurun_out/pmc_gbC.log; exit 1; }
echo done
