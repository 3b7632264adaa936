# GPU tests (all) then the DPS timings
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpujob_tests.sh tests > /dev/null; RC=$?
tail -3 gpurun_out/gpu_tests_sel.log
[ $RC -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gpu_tests_sel.log | head; exit 1; }
bash tools/gpujob_dps.sh
