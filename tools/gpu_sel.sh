cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "sel or sparse or pool or halo_wgrad" > gpurun_out/sel_pytest.log 2>&1 || { tail -40 gpurun_out/sel_pytest.log; exit 1; }
tail -2 gpurun_out/sel_pytest.log
timeout -k 10 300 python bench.py --groupby-extra 0 > gpurun_out/bench_cnn.json 2> gpurun_out/bench_cnn.err || { tail -30 gpurun_out/bench_cnn.err; exit 1; }
cat gpurun_out/bench_cnn.json
PTG_SPARSE_FIRST=0 timeout -k 10 300 python bench.py --groupby-extra 0 > gpurun_out/bench_cnn0.json 2>> gpurun_out/bench_cnn.err || exit 1
cat gpurun_out/bench_cnn0.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cnn -o run -- python bench.py --steps 10 --warmup 3 --groupby-extra 0 > gpurun_out/prof_cnn.log 2>&1 || exit 1
echo done
