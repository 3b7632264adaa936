# GroupNorm parameter-gradient partials folded into the backward statistics pass: parity, step time
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04r; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_unet_train.py tests/test_gpu_dps.py -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
grep -E "wide128|tiny16|worst|loss_rel" $O/tests.log | cut -c1-300 | head
timeout -k 10 300 python3 tools/kbench.py utrain --batch 16 --size 128 > $O/ut.out 2> $O/ut.err || { tail -20 $O/ut.err; exit 4; }
grep unet_train_step $O/ut.out | cut -c1-330
