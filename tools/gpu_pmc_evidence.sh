#!/bin/bash
# MFMA / LDS / HBM evidence for the CNN-B1 training step: three PMC passes (counter limits per pass:
# 8 SQ + 2 GRBM; FETCH_SIZE and WRITE_SIZE each alone), kernel-trace only.  tools/pmc_report.py
# turns them into per-kernel MFMA utilisation, LDS conflict rate and HBM bandwidth.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R && mkdir -p gpurun_out
WL=${WL:-cnn_b1}
ARGS="--workload $WL --steps 2 --warmup 1 --groupby-extra 0"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcE_${WL}_a -o run -- python bench.py $ARGS > gpurun_out/pmcE_${WL}_a.log 2>&1 || { tail -20 gpurun_out/pmcE_${WL}_a.log; exit 1; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcE_${WL}_b -o run -- python bench.py $ARGS > gpurun_out/pmcE_${WL}_b.log 2>&1 || { tail -20 gpurun_out/pmcE_${WL}_b.log; exit 1; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcE_${WL}_c -o run -- python bench.py $ARGS > gpurun_out/pmcE_${WL}_c.log 2>&1 || { tail -20 gpurun_out/pmcE_${WL}_c.log; exit 1; }
echo done
