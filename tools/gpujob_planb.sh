# small-batch planner experiment: U-Net forward at B = 1 (64^2 and config A's 32^2) under plan-batch / tile knobs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/planb; mkdir -p $O
for env in "CFD_PLAN_B=8" "CFD_PLAN_B=1" "CFD_PLAN_B=2" "CFD_PLAN_B=1 CFD_CONV_KH=0" "CFD_PLAN_B=1 CFD_CONV_NW8=0" "CFD_PLAN_B=1 CFD_CONV_TARGET_WG=1536" "CFD_PLAN_B=1 CFD_CONV_1X1_SPLIT=1" "CFD_PLAN_B=1 CFD_CONV_KH=0 CFD_CONV_NW8=0 CFD_CONV_1X1_SPLIT=1"; do
  for spec in "--size 64 --batch 1" "--size 32 --mult 1,2,3,4 --batch 1" "--size 64 --batch 2"; do
    r=$(env $env timeout -k 10 120 python3 tools/kbench.py unet $spec 2>/dev/null | tail -1) || { echo "FAIL $env $spec"; exit 1; }
    echo "$env | $spec | $r"
  done
done | tee $O/planb.log
