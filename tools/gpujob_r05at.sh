# round 5at: conv defaults CFD_CONV_PF 2 / CFD_CONV_XCD 4 -- whole GPU suite (knob bit-identity included), smoke,
# loop probe, the driver's bench command
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05at; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/gpu_tests.log | head; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
LOOP_MODES=2:4 timeout -k 10 300 python3 tools/loop_probe.py E100 B8 B1 A > $O/lp.out 2> $O/lp.err || { tail -20 $O/lp.err; exit 3; }
python3 -c "
import json
r=[json.loads(l) for l in open('$O/lp.out') if 'mode' in l]
print('HEAD', ' '.join('%s=%.3f' % (x['case'], x['ms_per_step']) for x in r))"
timeout -k 10 900 python3 bench.py --steps 20 --warmup 5 > $O/benchB20.json 2> $O/benchB20.err || { tail -20 $O/benchB20.err; exit 4; }
python3 -c "import json; d=json.load(open('$O/benchB20.json')); print('B20', round(d['value'],4), round(d['ms_per_step'],1), d['roofline']['frac'])"
