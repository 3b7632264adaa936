# Full GPU suite on the default build, then a same-box A/B of two in-tree builds
# (default vs CFD_LIB=libconfild_hip_base.so): U-Net forward (B = 8, split) and
# one config-D DPS step, 3 alternating rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error|error" gpurun_out/gpu_tests.log | tail -30; exit 1; }
tail -n 1 gpurun_out/gpu_tests.log
for r in 1 2 3; do
for V in "CFD_LIB=libconfild_hip.so" "CFD_LIB=libconfild_hip_base.so"; do
env $V timeout -k 10 200 python tools/kbench.py unet --unet-compute split_f16 > gpurun_out/kb_u.log 2>&1 || { cat gpurun_out/kb_u.log; exit 2; }
echo "$V $(grep kernel gpurun_out/kb_u.log | cut -c60-200)"
env $V timeout -k 10 200 python tools/kbench.py dps > gpurun_out/kb_d.log 2>&1 || { cat gpurun_out/kb_d.log; exit 2; }
echo "$V $(grep kernel gpurun_out/kb_d.log | cut -c1-300)"
done; done
