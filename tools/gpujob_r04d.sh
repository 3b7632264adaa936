# K1s register-ring depth: bit-identity and same-box timing at B=1 / config A / B=8
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_knobs.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
for PF in 1 2 3; do
for spec in "--size 64 --batch 1" "--size 32 --mult 1,2,3,4 --batch 1" "--size 64 --batch 8"; do
CFD_CONV_PF=$PF timeout -k 10 200 python tools/kbench.py unet $spec > $O/kb.log 2>&1 || { cat $O/kb.log; exit 2; }
echo "PF=$PF | $spec | $(grep kernel $O/kb.log | cut -c1-200)"
done; done; done
