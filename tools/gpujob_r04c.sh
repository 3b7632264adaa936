# A/B of the new library against the round's base build (same box), the K1s ring depth sweep,
# and the parity tests the changes touch
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_knobs.py tests/test_gpu_parity.py tests/test_gpu_unet_split.py "tests/test_gpu_cfg.py::test_configE_1000_step_segments" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for L in libconfild_hip.so libconfild_hip_base.so; do
for spec in "--size 64 --batch 8" "--size 64 --batch 1" "--size 32 --mult 1,2,3,4 --batch 1" "--size 128 --batch 8 --unet-compute bf16"; do
CFD_LIB=$L timeout -k 10 200 python tools/kbench.py unet $spec > $O/kb.log 2>&1 || { cat $O/kb.log; exit 2; }
echo "$L | $spec | $(grep kernel $O/kb.log | cut -c1-200)"
done; done
for PF in 2 3; do
for spec in "--size 64 --batch 1" "--size 32 --mult 1,2,3,4 --batch 1" "--size 64 --batch 8"; do
CFD_CONV_PF=$PF timeout -k 10 200 python tools/kbench.py unet $spec > $O/kb.log 2>&1 || { cat $O/kb.log; exit 2; }
echo "PF=$PF | $spec | $(grep kernel $O/kb.log | cut -c1-200)"
done; done; done
