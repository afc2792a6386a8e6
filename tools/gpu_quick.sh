#!/bin/bash
# Quick GPU pass: GPU tests + CNN-B1 bench (+ optional ResNet-50 bench with RN=1).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --groupby-extra 0 > gpurun_out/bench_cnn.json 2> gpurun_out/bench_cnn.err || { tail -30 gpurun_out/bench_cnn.err; exit 1; }
cat gpurun_out/bench_cnn.json
if [ "${RN:-0}" = "1" ]; then
timeout -k 10 400 python bench.py --workload resnet50 --batch-size 128 --steps 10 --warmup 3 > gpurun_out/bench_rn50.json 2> gpurun_out/bench_rn50.err || { tail -30 gpurun_out/bench_rn50.err; exit 1; }
cat gpurun_out/bench_rn50.json
fi
if [ "${PROF:-0}" = "1" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cnn -o run -- python bench.py --steps 10 --warmup 3 --groupby-extra 0 > gpurun_out/prof_cnn.log 2>&1 || exit 1
fi
echo done
