# Same-box sweep of environment settings ($SWEEP, space-separated VAR=value
# entries) over the U-Net forward kernel bench, 2 alternating rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
for V in $SWEEP; do
env $V timeout -k 10 200 python tools/kbench.py unet --unet-compute split_f16 > gpurun_out/kb_u.log 2>&1 || { cat gpurun_out/kb_u.log; exit 2; }
echo "$V $(grep -i ms gpurun_out/kb_u.log | tail -1 | cut -c60-160)"
done; done
