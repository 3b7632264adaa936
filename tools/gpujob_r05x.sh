# round 5 checkpoint x: whole GPU suite (release + debug), smoke, the default bench under a kernel trace,
# bench lines A / C / D / E / Case4 with their CPU baselines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/gpu_tests.log | head; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 bench.py > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 3; }
cat $O/bench_prof.json
S=$(find $O/prof_bench -name "*kernel_stats.csv" | head -1); cp $S $O/bench_kernel_stats.csv; rm -rf $O/prof_bench
timeout -k 10 400 python3 bench.py > $O/benchB.json 2> $O/benchB.err || { tail -20 $O/benchB.err; exit 4; }
timeout -k 10 300 python3 bench.py --config A --steps 5 --warmup 1 > $O/benchA.json 2> $O/benchA.err || { tail -20 $O/benchA.err; exit 5; }
timeout -k 10 300 python3 bench.py --config C > $O/benchC.json 2> $O/benchC.err || { tail -20 $O/benchC.err; exit 6; }
timeout -k 10 400 python3 bench.py --config E --steps 1 --warmup 0 > $O/benchE.json 2> $O/benchE.err || { tail -20 $O/benchE.err; exit 7; }
timeout -k 10 300 python3 bench.py --config D --steps 2 --warmup 1 > $O/benchD.json 2> $O/benchD.err || { tail -20 $O/benchD.err; exit 8; }
timeout -k 10 500 python3 bench.py --config Case4 --steps 1 --warmup 1 > $O/benchCase4.json 2> $O/benchCase4.err || { tail -20 $O/benchCase4.err; exit 9; }
for c in B A C E D Case4; do python3 -c "import json; d=json.load(open('$O/bench$c.json')); r=d.get('roofline') or {}; print('$c', round(d['value'],3), d['unit'], round(d['ms_per_step'],2), 'ms/step frac', r.get('frac'), 'cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value'],5))"; done
