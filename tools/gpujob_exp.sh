set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_siren_split.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/split_tests.log; exit 1; }
grep -E "sine|passed|failed" gpurun_out/split_tests.log | tail -5
