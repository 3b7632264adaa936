# round 5c: which switch changes bits (KV pack fusion / side stream / LDS epilogue)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python tools/dev/env_bits.py "" "CFD_ATTN_KVFUSE=0" "CFD_UNET_SIDE=0" "CFD_CONV_LDSEPI=0" "CFD_CONV_LDSEPI=0 CFD_ATTN_KVFUSE=0" "CFD_UNET_SIDE=0 CFD_ATTN_KVFUSE=0" || exit 1
rm -rf gpurun_out/envbits
