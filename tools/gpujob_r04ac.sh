# TrainLoop: bias gradients from the split weight-gradient kernel
# parity, same-box A/B against the previous library, kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ac; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_unet_train.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for spec in "libconfild_hip_prev.so 1" "libconfild_hip.so 1" "libconfild_hip.so 0"; do
set -- $spec
CFD_LIB=$1 CFD_WGRAD_THIN=$2 timeout -k 10 300 python3 tools/kbench.py utrain --batch 16 --size 128 > $O/ut.out 2> $O/ut.err || { tail -20 $O/ut.err; exit 4; }
echo "$1 THIN=$2 $(grep unet_train_step $O/ut.out | cut -c60-260)"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ut -o run -- python3 tools/kbench.py utrain --batch 16 --size 128 > $O/utp.out 2> $O/utp.err || { tail -20 $O/utp.err; exit 5; }
rm -f $O/ut/run_kernel_trace.csv
