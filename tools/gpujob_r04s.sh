# TrainLoop: GroupNorm parameter partials from the backward pass + thin-layer weight gradients;
# parity, then same-box A/B against the library before both (libconfild_hip_prev.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04s; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_unet_train.py -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
grep -E "worst" $O/tests.log | cut -c1-250 | head -5
for r in 1 2; do
for L in libconfild_hip_prev.so libconfild_hip.so; do
CFD_LIB=$L timeout -k 10 300 python3 tools/kbench.py utrain --batch 16 --size 128 > $O/ut.out 2> $O/ut.err || { tail -20 $O/ut.err; exit 4; }
echo "$L $(grep unet_train_step $O/ut.out | cut -c60-330)"
done; done
