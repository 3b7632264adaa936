# K1s LDS epilogue in row bands (bf16 tiles): bit-identity, config-E timing, stamps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_knobs.py tests/test_gpu_bf16.py tests/test_gpu_parity.py -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for EP in 1 0; do
CFD_CONV_LDSEPI=$EP timeout -k 10 200 python tools/kbench.py unet --size 128 --batch 8 --unet-compute bf16 > $O/kb.log 2>&1 || { cat $O/kb.log; exit 5; }
echo "LDSEPI=$EP | E | $(grep kernel $O/kb.log | cut -c60-200)"
done; done
CFD_LIB=libconfild_hip_stamps.so timeout -k 10 200 python tools/dev/stamps.py --size 128 --batch 8 --bf16 --detail 400 > $O/e128b8.txt 2>&1 || { tail -20 $O/e128b8.txt; exit 3; }
tail -4 $O/e128b8.txt
for SM in 64 128 256; do
CFD_WGRAD_SMAX=$SM CFD_WGRAD_TARGET=8192 timeout -k 10 300 python3 tools/kbench.py utrain --batch 16 --size 128 > $O/ut$SM.out 2> $O/ut$SM.err || { tail -20 $O/ut$SM.err; exit 4; }
echo "WGRAD_SMAX=$SM $(grep unet_train_step $O/ut$SM.out | cut -c1-330)"
done
