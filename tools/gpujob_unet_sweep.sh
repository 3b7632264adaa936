set -o pipefail
cd $GRAFT_REPO_ROOT
for BM in 64 128; do for T in 256 512 1024; do
CFD_CONV_BM=$BM CFD_CONV_TARGET_WG=$T timeout -k 10 200 python tools/kbench.py unet --unet-compute split_f16 > gpurun_out/kb_u.log 2>&1 || { cat gpurun_out/kb_u.log; exit 2; }
echo "BM=$BM T=$T $(grep kernel gpurun_out/kb_u.log)"
done; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_unet -o run -- python3 tools/kbench.py unet --unet-compute split_f16 > gpurun_out/prof_unet.log 2>&1 || exit 3
S=$(find gpurun_out/prof_unet -name "*kernel_stats.csv" | head -1); head -14 $S
