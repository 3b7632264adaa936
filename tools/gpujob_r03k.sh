# Round-3 late checkpoint: GPU suite (debug build included), smoke, config B bench (CPU baseline),
# configs A and E, kernel stats of the config-B command; each step under its own limit
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${TAG:-r03k}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" gpurun_out/$T/gpu_tests.log | head -20; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 2; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 600 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 3; }
cat gpurun_out/$T/bench.json
timeout -k 10 300 python3 bench.py --config A --steps 20 --warmup 2 > gpurun_out/$T/benchA.json 2> gpurun_out/$T/benchA.err || { tail -20 gpurun_out/$T/benchA.err; exit 4; }
cat gpurun_out/$T/benchA.json
timeout -k 10 400 python3 bench.py --config E --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/$T/benchE.json 2> gpurun_out/$T/benchE.err || { tail -20 gpurun_out/$T/benchE.err; exit 5; }
cat gpurun_out/$T/benchE.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/$T/prof.log 2>&1 || { tail -20 gpurun_out/$T/prof.log; exit 6; }
S=$(find gpurun_out/$T/prof -name "*kernel_stats.csv" | head -1); cp $S gpurun_out/$T/bench_kernel_stats.csv; rm -rf gpurun_out/$T/prof
echo done
