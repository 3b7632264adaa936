# round 5 final check aq: whole GPU suite, smoke and the driver's default bench command at HEAD
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05aq; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/gpu_tests.log | head; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('B default', round(d['value'],4), d['steps'], d['warmup'], round(d['ms_per_step'],1), d['roofline']['frac'], d['cpu_baseline']['value'])"
