#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_workloads_gpu.py -x -q -s > gpurun_out/pytest_wl.log 2>&1 || { tail -40 gpurun_out/pytest_wl.log; exit 1; }
grep -E "s$|passed|failed" gpurun_out/pytest_wl.log | tail -5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_km -o run -- python workloads/raw-spark/spark_checks/python_checks/spark_workload_to_cloud_k8s.py > gpurun_out/prof_km.log 2>&1 || exit 1
echo done
