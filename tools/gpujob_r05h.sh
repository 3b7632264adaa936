# round 5h: U-Net forward kernel traces at HEAD (B=8 / B=1 64^2, config A, config E) with the conv / GroupNorm plan log
# (config B), kernel traces of the U-Net forwards (B=8 / B=1 64^2, config A, config E)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05h; mkdir -p $O
for spec in "b64b8 --size 64 --batch 8" "b64b1 --size 64 --batch 1" "a32b1 --size 32 --mult 1,2,3,4 --batch 1" "e128b8 --size 128 --batch 8 --unet-compute bf16"; do
  set -- $spec; tag=$1; shift
  CFD_CONV_LOG=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$tag -o run -- python3 tools/kbench.py unet "$@" > $O/$tag.out 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 3; }
  grep kernel $O/$tag.out
  rm -f $O/prof_$tag/run_kernel_trace.csv.gz
done
