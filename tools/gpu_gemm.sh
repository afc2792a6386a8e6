#!/bin/bash
# GEMM-engine pass: GEMM/conv kernel tests, ResNet GPU tests, ResNet-50 layer bench + bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_nn_kernels_gpu.py tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread -k "gemm or conv or resnet or dgrad or wgrad or linear" > gpurun_out/gemm_pytest.log 2>&1 || { tail -40 gpurun_out/gemm_pytest.log; exit 1; }
tail -1 gpurun_out/gemm_pytest.log
timeout -k 10 300 python tools/rn50_layer_bench.py --only fwd,dgrad,wgrad > gpurun_out/rn50_layers.txt 2>&1 || { tail -20 gpurun_out/rn50_layers.txt; exit 1; }
tail -1 gpurun_out/rn50_layers.txt
timeout -k 10 400 python bench.py --workload resnet50 --batch-size 128 --steps 10 --warmup 3 > gpurun_out/bench_rn50.json 2> gpurun_out/bench_rn50.err || { tail -30 gpurun_out/bench_rn50.err; exit 1; }
cat gpurun_out/bench_rn50.json
echo done
