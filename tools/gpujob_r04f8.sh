# planner sweep at the final HEAD (environment only): split-K workgroup target, K1x split limits
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04f8; mkdir -p $O
for r in 1 2; do
for E in "CFD_CONV_TARGET_WG=768" "CFD_CONV_TARGET_WG=512" "CFD_CONV_TARGET_WG=1024" "CFD_CONV_KMIN=2" "CFD_CONV_SMAX=64"; do
for spec in "--size 64 --batch 8" "--size 64 --batch 1" "--size 32 --mult 1,2,3,4 --batch 1"; do
env $E timeout -k 10 200 python tools/kbench.py unet $spec > $O/kb.log 2>&1 || { cat $O/kb.log; exit 5; }
echo "$E | $spec | $(grep kernel $O/kb.log | cut -c60-170)"
done; done; done
