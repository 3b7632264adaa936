set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_siren_split.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/split_tests.log; exit 1; }
grep -E "max err" gpurun_out/split_tests.log | tail -12
for V in "CFD_SIREN_EXP=0" "CFD_SIREN_EXP=1" "CFD_SIREN_EXP=2" "CFD_SIREN_SPLIT32=0"; do
env $V timeout -k 10 200 python tools/kbench.py siren --latents 128 --compute split_f16 > gpurun_out/kb_v.log 2>&1 || { cat gpurun_out/kb_v.log; exit 2; }
echo "$V $(grep kernel gpurun_out/kb_v.log)"
done
