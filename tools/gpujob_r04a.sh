# round 4 first profile: B=1 / B=8 U-Net forward kernel traces with the conv plan log
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04a
for spec in "a32b1 --size 32 --mult 1,2,3,4 --batch 1" "b64b1 --size 64 --batch 1" "b64b8 --size 64 --batch 8"; do
  set -- $spec; tag=$1; shift
  CFD_CONV_LOG=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04a/prof_$tag -o run -- python3 tools/kbench.py unet "$@" > gpurun_out/r04a/$tag.out 2> gpurun_out/r04a/$tag.err || { tail -20 gpurun_out/r04a/$tag.err; exit 3; }
  T=$(find gpurun_out/r04a/prof_$tag -name "*kernel_trace.csv" | head -1); cp $T gpurun_out/r04a/${tag}_trace.csv
  S=$(find gpurun_out/r04a/prof_$tag -name "*kernel_stats.csv" | head -1); cp $S gpurun_out/r04a/${tag}_stats.csv
  rm -rf gpurun_out/r04a/prof_$tag
  cat gpurun_out/r04a/$tag.out
done
timeout -k 10 120 python3 tools/dev/optim_probe.py cuda cpu > gpurun_out/r04a/optim_probe.txt 2>&1 || exit 4
