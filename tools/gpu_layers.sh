#!/bin/bash
# Per-op CNN-B1 layer timings (+ the prelu/pool kernel tests) on one MI355X.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_nn_kernels_gpu.py -q -x -k "prelu_pool or halo" > gpurun_out/layers_pytest.log 2>&1 || { tail -30 gpurun_out/layers_pytest.log; exit 1; }
tail -2 gpurun_out/layers_pytest.log
PYTHONPATH=. timeout -k 10 300 python tools/cnn_layer_bench.py ${LAYER_ARGS:-} 2>&1 | tee gpurun_out/layers.log
