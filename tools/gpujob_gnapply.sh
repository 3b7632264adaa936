# Consumer-side GroupNorm (K3c, CFD_GN_APPLY=1) against the materialised path
# (CFD_GN_APPLY=0), same box: U-Net parity tests first, then alternating forward
# benches at config B (B=8 and B=1), config A (32^2 B=1) and config E (128^2 bf16 B=8).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_unet_split.py tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gn_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/gn_tests.log; exit 1; }
tail -1 gpurun_out/gn_tests.log
for r in 1 2; do
for V in CFD_GN_APPLY=0 CFD_GN_APPLY=1; do
for spec in "--batch 8" "--batch 1" "--batch 1 --size 32 --mult 1,2,3,4" "--batch 8 --size 128 --bf16"; do
env $V timeout -k 10 200 python tools/kbench.py unet $spec > gpurun_out/kb_u.log 2>&1 || { cat gpurun_out/kb_u.log; exit 2; }
echo "$V $spec $(grep -i ms gpurun_out/kb_u.log | tail -1 | cut -c1-200)"
done; done; done
