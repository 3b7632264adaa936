# U-Net tests, then a same-box A/B over up to four environment settings
# (AB_A .. AB_D) of the U-Net forward (B = 8, split) and a config-D DPS step.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_unet_split.py tests/test_gpu_dps.py tests/test_gpu_cfg.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error|error" gpurun_out/ab_tests.log | tail -30; exit 1; }
tail -n 1 gpurun_out/ab_tests.log
for r in 1 2 3; do
for V in "$AB_A" "$AB_B" "$AB_C" "$AB_D"; do
[ -z "$V" ] && continue
env $V timeout -k 10 200 python tools/kbench.py unet --unet-compute split_f16 > gpurun_out/kb_u.log 2>&1 || { cat gpurun_out/kb_u.log; exit 2; }
echo "$V $(grep kernel gpurun_out/kb_u.log | cut -c60-200)"
done; done
for V in "$AB_A" "$AB_B"; do
env $V timeout -k 10 200 python tools/kbench.py dps > gpurun_out/kb_d.log 2>&1 || { cat gpurun_out/kb_d.log; exit 2; }
echo "$V $(grep kernel gpurun_out/kb_d.log | cut -c1-300)"
done
