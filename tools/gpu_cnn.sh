#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_nn_kernels_gpu.py tests/test_models_gpu.py -x -q > gpurun_out/pytest_cnn.log 2>&1 || { tail -40 gpurun_out/pytest_cnn.log; exit 1; }
tail -1 gpurun_out/pytest_cnn.log
timeout -k 10 300 python bench.py --groupby-extra 0 > gpurun_out/bench_cnn.json 2> gpurun_out/bench_cnn.err || { tail -30 gpurun_out/bench_cnn.err; exit 1; }
cat gpurun_out/bench_cnn.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cnn -o run -- python bench.py --steps 10 --warmup 3 --groupby-extra 0 > gpurun_out/prof_cnn.log 2>&1 || exit 1
echo done
