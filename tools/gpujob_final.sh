# Round checkpoint: full GPU suite + smoke, bench lines for configs B (default),
# C, A, E, D, Case4, and the rocprofv3 kernel stats of the default command.
set -o pipefail
TAG=${TAG:-r02}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
O=gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error|error" $O/gpu_tests_$TAG.log | head -20; exit 1; }
tail -n 1 $O/gpu_tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { tail -20 $O/smoke_$TAG.log; exit 2; }
tail -n 1 $O/smoke_$TAG.log
timeout -k 10 600 python3 bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 3; }
cut -c1-400 $O/bench_$TAG.json
timeout -k 10 300 python3 bench.py --config C --steps 1 --warmup 1 --no-cpu-baseline > $O/benchC_$TAG.json 2> $O/benchC_$TAG.err || { tail -20 $O/benchC_$TAG.err; exit 4; }
timeout -k 10 200 python3 bench.py --config A --steps 5 --warmup 1 > $O/benchA_$TAG.json 2> $O/benchA_$TAG.err || { tail -20 $O/benchA_$TAG.err; exit 5; }
timeout -k 10 300 python3 bench.py --config E --steps 1 --warmup 0 > $O/benchE_$TAG.json 2> $O/benchE_$TAG.err || { tail -20 $O/benchE_$TAG.err; exit 6; }
timeout -k 10 200 python3 bench.py --config D --steps 2 --warmup 1 > $O/benchD_$TAG.json 2> $O/benchD_$TAG.err || { tail -20 $O/benchD_$TAG.err; exit 7; }
timeout -k 10 300 python3 bench.py --config Case4 --dps-steps 200 --steps 1 --warmup 1 > $O/benchCase4_$TAG.json 2> $O/benchCase4_$TAG.err || { tail -20 $O/benchCase4_$TAG.err; exit 8; }
for c in C A E D Case4; do python3 -c "import json,sys; d=json.load(open('$O/bench${c}_$TAG.json')); print('$c', round(d['value'],3), d['unit'], round(d['ms_per_step'],1), 'ms/step')"; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 9; }
S=$(find gpurun_out/prof_final -name "*kernel_stats.csv" | head -1); cp $S $O/${TAG}_bench_kernel_stats.csv; head -8 $S | cut -c1-150
echo done
