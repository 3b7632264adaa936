# config-E forward kernel trace; TrainLoop with the one-atomic-per-workgroup gn_act
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04h; mkdir -p $O
CFD_CONV_LOG=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/e128 -o run -- python3 tools/kbench.py unet --size 128 --batch 8 --unet-compute bf16 > $O/e128.out 2> $O/e128.err || { tail -20 $O/e128.err; exit 3; }
grep kernel $O/e128.out
for W in 1 0; do
CFD_WGRAD_SPLIT=$W timeout -k 10 300 python3 tools/kbench.py utrain --batch 16 --size 128 > $O/ut$W.out 2> $O/ut$W.err || { tail -20 $O/ut$W.err; exit 4; }
echo "WGRAD_SPLIT=$W $(grep unet_train_step $O/ut$W.out | cut -c1-400)"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet_train.py -x -q --timeout 300 --timeout-method thread > $O/train_tests.log 2>&1 || { echo TRAINFAIL; tail -30 $O/train_tests.log; exit 5; }
tail -1 $O/train_tests.log
