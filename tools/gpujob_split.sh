set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_siren_split.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/split_tests.log; exit 1; }
grep -E "max err|PASS|FAIL" gpurun_out/split_tests.log | tail -3
CFD_SIREN_RB=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_siren_split.py -x -q --timeout 120 --timeout-method thread > gpurun_out/split_tests_rb1.log 2>&1 || { echo TESTFAIL RB1; tail -40 gpurun_out/split_tests_rb1.log; exit 1; }
for V in "CFD_SIREN_RB=1" "CFD_SIREN_RB=2" "CFD_SIREN_SPLIT_CG=2 CFD_SIREN_RB=2"; do
env $V timeout -k 10 200 python tools/kbench.py siren --latents 256 --compute split_f16 > gpurun_out/kb_v.log 2>&1 || { cat gpurun_out/kb_v.log; exit 2; }
echo "$V"; grep kernel gpurun_out/kb_v.log
done
