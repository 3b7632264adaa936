set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_unet -o run -- python3 tools/kbench.py unet --unet-compute split_f16 > gpurun_out/prof_unet.log 2>&1 || exit 3
S=$(find gpurun_out/prof_unet -name "*kernel_stats.csv" | head -1); cat $S
