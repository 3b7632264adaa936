# weight-gradient slices sized to whole rounds of resident blocks: TrainLoop step, parity
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04p; mkdir -p $O
for T in 512 1024 2048; do
CFD_WGRAD_TARGET=$T timeout -k 10 300 python3 tools/kbench.py utrain --batch 16 --size 128 > $O/ut$T.out 2> $O/ut$T.err || { tail -20 $O/ut$T.err; exit 4; }
echo "WGRAD_TARGET=$T $(grep unet_train_step $O/ut$T.out | cut -c1-330)"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet_train.py -x -q --timeout 300 --timeout-method thread > $O/train_tests.log 2>&1 || { echo TRAINFAIL; tail -30 $O/train_tests.log; exit 5; }
tail -1 $O/train_tests.log
