#!/bin/bash
# Full GPU pass: all GPU tests, headline bench (CNN-B1 + groupBy extra), ResNet-50 bench, rocprof of
# CNN-B1, ResNet-50 and groupBy.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench_cnn.json 2> gpurun_out/bench_cnn.err || { tail -30 gpurun_out/bench_cnn.err; exit 1; }
cat gpurun_out/bench_cnn.json
timeout -k 10 400 python bench.py --workload resnet50 --batch-size ${B:-128} --steps 10 --warmup 3 > gpurun_out/bench_rn50.json 2> gpurun_out/bench_rn50.err || { tail -30 gpurun_out/bench_rn50.err; exit 1; }
cat gpurun_out/bench_rn50.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cnn -o run -- python bench.py --steps 10 --warmup 3 --groupby-extra 0 > gpurun_out/prof_cnn.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rn50 -o run -- python bench.py --workload resnet50 --batch-size ${B:-128} --steps 5 --warmup 2 > gpurun_out/prof_rn50.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gb -o run -- python bench.py --workload groupby --steps 3 --warmup 1 > gpurun_out/prof_gb.log 2>&1 || exit 1
echo done
