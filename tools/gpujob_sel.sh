# selected GPU tests (args: pytest node ids), verbose with prints
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/sel_tests.log 2>&1
RC=$?
grep -E "PASS|FAIL|Error|error|config|drift|vs |subset" gpurun_out/sel_tests.log | tail -40
tail -3 gpurun_out/sel_tests.log
exit $RC
