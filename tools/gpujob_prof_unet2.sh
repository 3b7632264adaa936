# U-Net forward kernel trace with the convolution shape log (development)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export CFD_CONV_LOG=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_unet2 -o run -- python3 tools/kbench.py unet --unet-compute split_f16 > gpurun_out/prof_unet2.log 2> gpurun_out/prof_unet2.err || { tail gpurun_out/prof_unet2.err; exit 3; }
grep -c CONV gpurun_out/prof_unet2.err
