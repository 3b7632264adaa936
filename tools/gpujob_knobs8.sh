# planner knob sweep at config B (64^2, B = 8, split-f16) and config E (128^2, B = 8, bf16)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/knobs8; mkdir -p $O
for env in "CFD_X=0" "CFD_CONV_NW8=0" "CFD_CONV_NW8=1" "CFD_CONV_1X1_SPLIT=1" "CFD_CONV_NW8=0 CFD_CONV_1X1_SPLIT=1" "CFD_CONV_TARGET_WG=1536" "CFD_CONV_NW8=0 CFD_CONV_TARGET_WG=1536" "CFD_CONV_XCD=3" "CFD_X=0"; do
  for spec in "--size 64 --batch 8" "--size 128 --batch 8 --bf16"; do
    r=$(env $env timeout -k 10 120 python3 tools/kbench.py unet $spec 2>/dev/null | tail -1) || { echo "FAIL $env $spec"; exit 1; }
    echo "$env | $spec | $r"
  done
done | tee $O/knobs8.log
