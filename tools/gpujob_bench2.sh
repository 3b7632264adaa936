# Round-2 bench: default config-B line (with CPU baseline), config C at N=1,
# rocprofv3 kernel stats of the default command.
set -o pipefail
TAG=${TAG:-r02}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/profiles_new
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 14; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 python3 bench.py --config C --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/benchC_$TAG.json 2> gpurun_out/benchC_$TAG.err || { tail -20 gpurun_out/benchC_$TAG.err; exit 16; }
cat gpurun_out/benchC_$TAG.json
if [ -z "$NOPROF" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || { tail -20 gpurun_out/prof_bench.log; exit 15; }
S=$(find gpurun_out/prof_bench -name "*kernel_stats.csv" | head -1); cp $S gpurun_out/profiles_new/${TAG}_bench_kernel_stats.csv; head -14 $S
fi
echo done
