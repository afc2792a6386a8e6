#!/bin/bash
# ResNet-50 pass: resnet/graph GPU tests, bench (b128) and its rocprof kernel stats.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_resnet_gpu.py tests/test_graph_capture_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/rn_pytest.log 2>&1 || { tail -40 gpurun_out/rn_pytest.log; exit 1; }
tail -1 gpurun_out/rn_pytest.log
timeout -k 10 400 python bench.py --workload resnet50 --batch-size 128 --steps 10 --warmup 3 > gpurun_out/bench_rn50.json 2> gpurun_out/bench_rn50.err || { tail -30 gpurun_out/bench_rn50.err; exit 1; }
cat gpurun_out/bench_rn50.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rn50 -o run -- python bench.py --workload resnet50 --batch-size 128 --steps 5 --warmup 2 > gpurun_out/prof_rn50.log 2>&1 || exit 1
echo done
