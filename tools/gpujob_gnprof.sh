# Kernel statistics of single U-Net forwards (config B, B=8 and B=1) under two
# environment settings (PA / PB), for tools/kstats.py comparisons.  SPECS: ";"-separated
# "tag kbench-args" entries (default config B at B=8 and B=1).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gp
for V in "${PA:-CFD_GN_APPLY=0}" "${PB:-CFD_GN_APPLY=1}"; do
IFS=";" read -ra SPECS <<< "${SPECS:-b8 --batch 8;b1 --batch 1}"
for spec in "${SPECS[@]}"; do
  set -- $spec; tag=$1_${V//[^A-Za-z0-9]/_}; shift
  export $V
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gp/prof_$tag -o run -- python3 tools/kbench.py unet "$@" > gpurun_out/gp/$tag.out 2> gpurun_out/gp/$tag.err || { tail -20 gpurun_out/gp/$tag.err; exit 3; }
  S=$(find gpurun_out/gp/prof_$tag -name "*kernel_stats.csv" | head -1); cp $S gpurun_out/gp/${tag}_stats.csv
  rm -rf gpurun_out/gp/prof_$tag
  echo "$tag $(cat gpurun_out/gp/$tag.out)"
  unset ${V%%=*}
done; done
