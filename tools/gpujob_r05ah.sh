# round 5 checkpoint ah: whole GPU suite, smoke, the driver's bench command under a kernel trace (pipelined B),
# the same without the trace, D and Case4 lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ah; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/gpu_tests.log | head; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 bench.py --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 3; }
S=$(find $O/prof_bench -name "*kernel_stats.csv" | head -1); cp $S $O/bench_kernel_stats.csv; rm -rf $O/prof_bench
python3 -c "import json; d=json.load(open('$O/bench_prof.json')); print('B(prof)', round(d['value'],4), round(d['ms_per_step'],1), d['roofline']['launch_ms'], d['roofline']['frac'])"
timeout -k 10 900 python3 bench.py --steps 20 --warmup 5 > $O/benchB20.json 2> $O/benchB20.err || { tail -20 $O/benchB20.err; exit 4; }
python3 -c "import json; d=json.load(open('$O/benchB20.json')); print('B20', round(d['value'],4), round(d['ms_per_step'],1), d['roofline']['frac'])"
timeout -k 10 300 python3 bench.py --config D --steps 2 --warmup 1 > $O/benchD.json 2> $O/benchD.err || { tail -20 $O/benchD.err; exit 8; }
timeout -k 10 500 python3 bench.py --config Case4 --steps 1 --warmup 1 > $O/benchCase4.json 2> $O/benchCase4.err || { tail -20 $O/benchCase4.err; exit 9; }
for c in D Case4; do python3 -c "import json; d=json.load(open('$O/bench$c.json')); print('$c', round(d['value'],3), d['unit'], round(d['ms_per_step'],2), 'cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value'],5))"; done
