#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_resnet_gpu.py tests/test_nn_kernels_gpu.py -x -q > gpurun_out/pytest_resnet.log 2>&1 || { tail -40 gpurun_out/pytest_resnet.log; exit 1; }
tail -1 gpurun_out/pytest_resnet.log
timeout -k 10 400 python bench.py --workload resnet50 --batch-size 128 --steps 10 --warmup 3 > gpurun_out/bench_rn50.json 2> gpurun_out/bench_rn50.err || { tail -30 gpurun_out/bench_rn50.err; exit 1; }
cat gpurun_out/bench_rn50.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rn50 -o run -- python bench.py --workload resnet50 --batch-size 128 --steps 5 --warmup 2 > gpurun_out/prof_rn50.log 2>&1 || exit 1
echo done
