# round-4 checkpoint benches: the default bench under a kernel trace (roofline cross-check),
# then every configuration with its cpu_baseline, each under its own limit
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 bench.py > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 2; }
cat $O/bench_prof.json
rm -f $O/prof_bench/run_kernel_trace.csv
for cfg in B A C D E; do
  timeout -k 10 600 python bench.py --config $cfg > $O/bench$cfg.json 2> $O/bench$cfg.err || { echo BENCHFAIL $cfg; tail -20 $O/bench$cfg.err; exit 3; }
  cat $O/bench$cfg.json
done
timeout -k 10 600 python bench.py --config Case4 --dps-steps 1000 > $O/benchCase4.json 2> $O/benchCase4.err || { echo BENCHFAIL Case4; tail -20 $O/benchCase4.err; exit 3; }
cat $O/benchCase4.json
