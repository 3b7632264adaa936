# A/B of the K1x split-K limits (CFD_CONV_KMIN / CFD_CONV_SMAX; shipped 4 / 32, before 8 / 16):
# U-Net forward at config A (32^2 B=1), B=1 64^2 and B=8 64^2, two interleaved rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
for round in 1 2; do
for env in "CFD_CONV_KMIN=8 CFD_CONV_SMAX=16" "CFD_X=0" "CFD_CONV_KMIN=2 CFD_CONV_SMAX=64"; do
  for spec in "--size 32 --mult 1,2,3,4 --batch 1" "--size 64 --batch 1" "--size 64 --batch 8"; do
    echo -n "$env | $spec | "
    env $env timeout -k 10 200 python3 tools/kbench.py unet $spec 2>/dev/null | tail -1 || exit 2
  done
done
done
