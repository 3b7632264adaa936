# GPU suite + smoke only (round checkpoint of parity)
set -o pipefail
TAG=${TAG:-r03}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error|error" gpurun_out/gpu_tests_$TAG.log | head -20; tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 2; }
tail -1 gpurun_out/smoke_$TAG.log
