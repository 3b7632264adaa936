# Same-box A/B of one build under two environment settings (AB_A / AB_B), after
# the U-Net GPU parity tests: 3 alternating rounds of the U-Net forward kernel bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_unet_split.py tests/test_gpu_dps.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for r in 1 2 3; do
for V in "$AB_A" "$AB_B"; do
env $V timeout -k 10 200 python tools/kbench.py unet --unet-compute split_f16 > gpurun_out/kb_u.log 2>&1 || { cat gpurun_out/kb_u.log; exit 2; }
echo "$V $(grep -i ms gpurun_out/kb_u.log | tail -1 | cut -c1-200)"
done; done
