# config-E path: bf16 GPU tests, then a same-box A/B of the 128^2 bf16 U-Net
# forward (B = 8) with and without the bf16 halo-tile convolutions (K1hb)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/bf16_tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error|error|err" gpurun_out/bf16_tests.log | tail -30; exit 1; }
grep -E "err|PASS" gpurun_out/bf16_tests.log | cut -c1-200 | tail -12
for r in 1 2; do
for V in CFD_CONV_KHB=1 CFD_CONV_KHB=0; do
env $V timeout -k 10 200 python tools/kbench.py unet --size 128 --unet-compute bf16 > gpurun_out/kb_u.log 2>&1 || { cat gpurun_out/kb_u.log; exit 2; }
echo "$V $(grep kernel gpurun_out/kb_u.log | cut -c40-200)"
done; done
