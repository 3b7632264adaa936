# TrainLoop kernel trace at HEAD (Case1 recipe)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ut -o run -- python3 tools/kbench.py utrain --batch 16 --size 128 > $O/ut.out 2> $O/ut.err || { tail -20 $O/ut.err; exit 4; }
grep unet_train_step $O/ut.out | cut -c1-300
rm -f $O/ut/run_kernel_trace.csv
