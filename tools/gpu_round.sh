#!/bin/bash
# One GPU pass: kernel tests, bench at the default and b256, rocprof kernel stats of the bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -30 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
timeout -k 10 300 python bench.py --batch-size 256 > gpurun_out/bench_b256.json 2>>gpurun_out/bench_default.err || exit 1
cat gpurun_out/bench_b256.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cnn -o run -- python bench.py --steps 10 --warmup 3 > gpurun_out/prof_cnn.log 2>&1 || exit 1
echo done
