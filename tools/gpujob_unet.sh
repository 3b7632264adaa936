set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_unet_split.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/unet_split_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/unet_split_tests.log; exit 1; }
grep -E "max\|err|PASS|FAIL" gpurun_out/unet_split_tests.log
for C in fp32 split_f16; do
timeout -k 10 200 python tools/kbench.py unet --unet-compute $C > gpurun_out/kb_u.log 2>&1 || { cat gpurun_out/kb_u.log; exit 2; }
grep kernel gpurun_out/kb_u.log
done
