# Round-end evidence on one MI355X: the whole GPU suite (debug build included),
# smoke(), and the default bench line, each step under its own time limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/final/gpu_tests.log; exit 1; }
tail -1 gpurun_out/final/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/final/smoke.log; exit 2; }
tail -1 gpurun_out/final/smoke.log
if [ -n "$WITH_BENCH" ]; then
timeout -k 10 600 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { echo BENCHFAIL; tail -20 gpurun_out/final/bench.err; exit 3; }
cat gpurun_out/final/bench.json
fi
