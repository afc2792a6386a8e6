#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_graph_capture_gpu.py -x -q -s > gpurun_out/pytest_graph.log 2>&1 || { tail -40 gpurun_out/pytest_graph.log; exit 1; }
grep -E "steps/s|passed|failed" gpurun_out/pytest_graph.log
timeout -k 10 300 python bench.py --groupby-extra 0 --graph 1 > gpurun_out/bench_cnn_graph.json 2> gpurun_out/bench_cnn_graph.err || { tail -30 gpurun_out/bench_cnn_graph.err; exit 1; }
cat gpurun_out/bench_cnn_graph.json
timeout -k 10 300 python bench.py --workload resnet50 --batch-size 128 --steps 10 --warmup 3 --graph 1 > gpurun_out/bench_rn50_graph.json 2> gpurun_out/bench_rn50_graph.err || { tail -30 gpurun_out/bench_rn50_graph.err; exit 1; }
cat gpurun_out/bench_rn50_graph.json
echo done
