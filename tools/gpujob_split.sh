set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_siren_split.py tests/test_gpu_parity.py -k "siren or trainer" -x -v -s --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/split_tests.log; exit 1; }
grep -E "max err|PASS|FAIL" gpurun_out/split_tests.log
timeout -k 10 200 python tools/kbench.py siren --latents 512 --compute split_f16 > gpurun_out/kb_split.log 2>&1 || { cat gpurun_out/kb_split.log; exit 2; }
timeout -k 10 200 python tools/kbench.py siren --latents 512 --compute f32 > gpurun_out/kb_f32.log 2>&1 || exit 3
cat gpurun_out/kb_split.log gpurun_out/kb_f32.log
