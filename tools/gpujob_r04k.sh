# full GPU suite at HEAD (release + debug builds), smoke; TrainLoop step; stamps with epilogue ends
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 1300 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/gpu_tests.log | head; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -2 $O/smoke.log
timeout -k 10 300 python3 tools/kbench.py utrain --batch 16 --size 128 > $O/ut.out 2> $O/ut.err || { tail -20 $O/ut.err; exit 4; }
grep unet_train_step $O/ut.out | cut -c1-400
CFD_LIB=libconfild_hip_stamps.so timeout -k 10 200 python tools/dev/stamps.py --size 128 --batch 8 --bf16 --detail 400 > $O/e128b8.txt 2>&1 || { tail -20 $O/e128b8.txt; exit 3; }
tail -4 $O/e128b8.txt
