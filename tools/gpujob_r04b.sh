# round 4 checkpoint: whole GPU suite (debug build included), smoke, every bench
# configuration with its cpu_baseline, each step under its own limit
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/gpu_tests.log | head; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
for cfg in B A C D E; do
  timeout -k 10 600 python bench.py --config $cfg > $O/bench$cfg.json 2> $O/bench$cfg.err || { echo BENCHFAIL $cfg; tail -20 $O/bench$cfg.err; exit 3; }
  cat $O/bench$cfg.json
done
timeout -k 10 600 python bench.py --config Case4 --dps-steps 1000 > $O/benchCase4.json 2> $O/benchCase4.err || { echo BENCHFAIL Case4; tail -20 $O/benchCase4.err; exit 3; }
cat $O/benchCase4.json
