# GPU test subset (or all with no args), verbose with prints, one process
set -o pipefail
cd $GRAFT_REPO_ROOT
ARGS=${@:-tests}
timeout -k 10 900 python -u -m pytest $ARGS -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_sel.log 2>&1
RC=$?
grep -E "PASS|FAIL|Error|error|drift|vs reference|config|Case4|U-Net" gpurun_out/gpu_tests_sel.log | tail -60
tail -3 gpurun_out/gpu_tests_sel.log
exit $RC
