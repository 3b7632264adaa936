# GroupNorm wave-butterfly reduction, float-reciprocal pixel-table division, split
# weight-gradient LDS layout: parity, in-kernel stamps, same-box A/B vs the round's
# base library, TrainLoop step (split vs fp32 weight-gradient products)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_knobs.py tests/test_gpu_unet_split.py tests/test_gpu_bf16.py "tests/test_gpu_cfg.py::test_configE_100_consecutive_steps" -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
grep -E "100 steps" $O/tests.log
CFD_LIB=libconfild_hip_stamps.so timeout -k 10 200 python tools/dev/stamps.py --size 64 --batch 1 --detail 400 --json $O/b64b1.json > $O/b64b1.txt 2>&1 || { tail -20 $O/b64b1.txt; exit 2; }
tail -6 $O/b64b1.txt
for r in 1 2; do
for L in libconfild_hip_base.so libconfild_hip.so; do
for spec in "--size 64 --batch 1" "--size 32 --mult 1,2,3,4 --batch 1" "--size 64 --batch 8"; do
CFD_LIB=$L timeout -k 10 200 python tools/kbench.py unet $spec > $O/kb.log 2>&1 || { cat $O/kb.log; exit 5; }
echo "$L | $spec | $(grep kernel $O/kb.log | cut -c60-200)"
done; done; done
for r in 1 2; do
for SN in 1 257 513; do
for spec in "--size 64 --batch 8" "--size 64 --batch 4" "--size 32 --mult 1,2,3,4 --batch 8"; do
CFD_CONV_SMALLN=$SN timeout -k 10 200 python tools/kbench.py unet $spec > $O/kb.log 2>&1 || { cat $O/kb.log; exit 5; }
echo "SMALLN=$SN | $spec | $(grep kernel $O/kb.log | cut -c60-200)"
done; done; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet_train.py -x -v -s --timeout 300 --timeout-method thread > $O/train_tests.log 2>&1 || { echo TRAINFAIL; grep -E "FAIL|Error|assert" $O/train_tests.log | head -20; tail -30 $O/train_tests.log; exit 3; }
tail -1 $O/train_tests.log
grep -E "wide128|worst|excess" $O/train_tests.log | head
for W in 1 0; do
CFD_WGRAD_SPLIT=$W timeout -k 10 300 python tools/kbench.py utrain --batch 16 --size 128 > $O/utrain$W.log 2>&1 || { tail -20 $O/utrain$W.log; exit 4; }
echo "WGRAD_SPLIT=$W $(grep unet_train_step $O/utrain$W.log | cut -c1-400)"
done
