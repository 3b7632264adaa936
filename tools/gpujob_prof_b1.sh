# kernel traces of single U-Net forwards at small batch (config A 32^2 B=1, config B 64^2 B=1 and B=8)
# with the convolution plan log, for tools/convjoin.py / tools/kstats.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/b1
for spec in "a32b1 --size 32 --mult 1,2,3,4 --batch 1" "b64b1 --size 64 --batch 1" "b64b8 --size 64 --batch 8" ${EXTRA_SPECS}; do
  set -- $spec; tag=$1; shift
  CFD_CONV_LOG=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b1/prof_$tag -o run -- python3 tools/kbench.py unet "$@" > gpurun_out/b1/$tag.out 2> gpurun_out/b1/$tag.err || { tail -20 gpurun_out/b1/$tag.err; exit 3; }
  T=$(find gpurun_out/b1/prof_$tag -name "*kernel_trace.csv" | head -1); cp $T gpurun_out/b1/${tag}_trace.csv
  S=$(find gpurun_out/b1/prof_$tag -name "*kernel_stats.csv" | head -1); cp $S gpurun_out/b1/${tag}_stats.csv
  rm -rf gpurun_out/b1/prof_$tag
  cat gpurun_out/b1/$tag.out
done
