# kernel traces of B=1 U-Net forwards (64^2) under the small-batch planner knobs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/b1p
for spec in "p1 CFD_PLAN_B=1" "p1nw CFD_PLAN_B=1 CFD_CONV_NW8=0 CFD_CONV_KH=0"; do
  set -- $spec; tag=$1; shift
  env "$@" CFD_CONV_LOG=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/b1p/prof_$tag -o run -- python3 tools/kbench.py unet --size 64 --batch 1 > gpurun_out/b1p/$tag.out 2> gpurun_out/b1p/$tag.err || { tail -20 gpurun_out/b1p/$tag.err; exit 3; }
  T=$(find gpurun_out/b1p/prof_$tag -name "*kernel_trace.csv" | head -1); cp $T gpurun_out/b1p/${tag}_trace.csv
  rm -rf gpurun_out/b1p/prof_$tag
  cat gpurun_out/b1p/$tag.out
done
