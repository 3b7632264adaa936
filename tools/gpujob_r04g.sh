# K1h / K1hb split-K 2 as in-workgroup K groups: bit-identity (knob test), timings
# against the slab path; TrainLoop kernel trace, split vs fp32 weight gradients
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_knobs.py tests/test_gpu_parity.py tests/test_gpu_bf16.py -x -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for KG in 128 0 1; do
for spec in "--size 64 --batch 8" "--size 64 --batch 1" "--size 32 --mult 1,2,3,4 --batch 8" "--size 128 --batch 8 --unet-compute bf16"; do
CFD_CONV_KHG=$KG timeout -k 10 200 python tools/kbench.py unet $spec > $O/kb.log 2>&1 || { cat $O/kb.log; exit 5; }
echo "KHG=$KG | $spec | $(grep kernel $O/kb.log | cut -c60-200)"
done; done; done
for W in 1 0; do
CFD_WGRAD_SPLIT=$W timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ut$W -o run -- python3 tools/kbench.py utrain --batch 16 --size 128 > $O/ut$W.out 2> $O/ut$W.err || { tail -20 $O/ut$W.err; exit 4; }
echo "WGRAD_SPLIT=$W $(grep unet_train_step $O/ut$W.out | cut -c1-300)"
done
