#!/bin/bash
# sparse pool record on layers 2-3: tests, gantt, A/B at b256 and b32
set -o pipefail
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_nn_kernels_gpu.py -m gpu \
  -k "sparse or dgrad or conv" > gpurun_out/t_sp.log 2>&1 || { tail -30 gpurun_out/t_sp.log; exit 1; }
tail -1 gpurun_out/t_sp.log
PTG_SPARSE_POOL=1 BENCH_ARGS="--batch-size 256" bash tools/gpu.sh prof > /dev/null || exit 1
python tools/step_gantt.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv > gpurun_out/gantt_sp.txt 2>&1
rm -rf gpurun_out/prof_cnn_b1
ABM_ENVS="PTG_SPARSE_POOL=1" bash tools/gpu.sh abm || exit 1
ABM_ENVS="PTG_SPARSE_POOL=1" BENCH_ARGS="--batch-size 32" bash tools/gpu.sh abm || exit 1
ABM_ENVS="PTG_SPARSE_POOL=1" BENCH_ARGS="--batch-size 64" bash tools/gpu.sh abm
