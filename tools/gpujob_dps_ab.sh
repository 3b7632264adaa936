# DPS GPU tests (split-f16 input-VJP), then a same-box A/B of the DPS step:
# split-f16 transposed convolutions (default) vs fp32 (CFD_VJP_SPLIT=0).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dps.py tests/test_gpu_e2e.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dps_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/dps_tests.log; exit 1; }
tail -1 gpurun_out/dps_tests.log
for r in 1 2; do
for V in CFD_VJP_SPLIT=1 CFD_VJP_SPLIT=0; do
env $V timeout -k 10 200 python tools/kbench.py dps > gpurun_out/kb_d.log 2>&1 || { cat gpurun_out/kb_d.log; exit 2; }
echo "$V $(tail -1 gpurun_out/kb_d.log | cut -c1-400)"
done; done
