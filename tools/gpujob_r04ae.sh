# kept GroupNorm outputs in the training tape on / off, same box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ae; mkdir -p $O
for r in 1 2; do
for G in 1 0; do
CFD_TAPE_GNOUT=$G timeout -k 10 300 python3 tools/kbench.py utrain --batch 16 --size 128 > $O/ut.out 2> $O/ut.err || { tail -20 $O/ut.err; exit 4; }
echo "TAPE_GNOUT=$G $(grep unet_train_step $O/ut.out | cut -c60-300)"
done; done
CFD_TAPE_GNOUT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p1 -o run -- python3 tools/kbench.py utrain --batch 16 --size 128 > $O/p1.out 2> $O/p1.err || exit 5
CFD_TAPE_GNOUT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p0 -o run -- python3 tools/kbench.py utrain --batch 16 --size 128 > $O/p0.out 2> $O/p0.err || exit 5
rm -f $O/p1/run_kernel_trace.csv $O/p0/run_kernel_trace.csv
