# A/B of two in-tree builds in one job (same box): CFD_LIB=libconfild_hip_old.so vs default
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
for L in libconfild_hip.so libconfild_hip_old.so; do
CFD_LIB=$L timeout -k 10 200 python tools/kbench.py unet --unet-compute split_f16 > gpurun_out/kb_u.log 2>&1 || { cat gpurun_out/kb_u.log; exit 2; }
echo "$L $(grep kernel gpurun_out/kb_u.log)"
done; done
