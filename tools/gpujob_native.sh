# native loop: GPU tests + timing probe
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_native_loop.py tests/test_gpu_e2e.py tests/test_gpu_unet_split.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/native_tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error|error|assert" gpurun_out/native_tests.log | head -30; tail -30 gpurun_out/native_tests.log; exit 1; }
tail -2 gpurun_out/native_tests.log
timeout -k 10 400 python -u tools/loop_probe.py > gpurun_out/loop_probe.log 2>&1 || { tail -30 gpurun_out/loop_probe.log; exit 2; }
cat gpurun_out/loop_probe.log
