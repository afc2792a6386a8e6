cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for wl in mnist cnn_a1 mlp; do
  timeout -k 10 200 python bench.py --workload $wl --groupby-extra 0 > gpurun_out/bench_$wl.json 2>gpurun_out/bench_$wl.err || { tail -5 gpurun_out/bench_$wl.err; exit 1; }
  cut -c1-260 gpurun_out/bench_$wl.json
  timeout -k 10 200 python bench.py --workload $wl --groupby-extra 0 --graph 1 > gpurun_out/bench_${wl}_g.json 2>>gpurun_out/bench_$wl.err || { tail -5 gpurun_out/bench_$wl.err; exit 1; }
  cut -c1-200 gpurun_out/bench_${wl}_g.json
done
