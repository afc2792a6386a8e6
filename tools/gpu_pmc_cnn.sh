#!/bin/bash
# PMC counters over a short CNN-B1 bench (kernel-trace only; two passes of <= 8 SQ counters).
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R && mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc_cnnA -o run -- python bench.py --steps 3 --warmup 1 --groupby-extra 0 > gpurun_out/pmc_cnnA.log 2>&1 || { tail -20 gpurun_out/pmc_cnnA.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LEVEL_WAVES SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_cnnB -o run -- python bench.py --steps 3 --warmup 1 --groupby-extra 0 > gpurun_out/pmc_cnnB.log 2>&1 || { tail -20 gpurun_out/pmc_cnnB.log; exit 1; }
echo done
