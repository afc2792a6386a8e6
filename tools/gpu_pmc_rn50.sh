#!/bin/bash
# PMC counters of the ResNet-50 conv GEMMs (rn50_layer_bench), kernel-trace only.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R && mkdir -p gpurun_out
export PYTHONPATH=$R
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_rn -o run -- python tools/rn50_layer_bench.py --iters 2 --only ${ONLY:-fwd,wgrad,dgrad} > gpurun_out/pmc_rn.log 2>&1 || { tail -20 gpurun_out/pmc_rn.log; exit 1; }
echo done
