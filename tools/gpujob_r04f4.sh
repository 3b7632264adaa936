# round-end U-Net PMC record (config B forward, 64^2 B=8): four counter passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=r04f4 bash tools/gpujob_pmc_unet_head.sh > /dev/null || exit 21
head -5 gpurun_out/r04f4_unet_pmc.txt
