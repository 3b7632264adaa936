# A/B of two in-tree builds in one job (same box): default vs CFD_LIB=libconfild_hip_old.so
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_unet_split.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for r in 1 2 3; do
for V in "CFD_LIB=libconfild_hip.so" "CFD_LIB=libconfild_hip_old.so" ${AB_EXTRA}; do
env $V timeout -k 10 200 python tools/kbench.py unet --unet-compute split_f16 > gpurun_out/kb_u.log 2>&1 || { cat gpurun_out/kb_u.log; exit 2; }
echo "$V $(grep kernel gpurun_out/kb_u.log | cut -c60-200)"
done; done
