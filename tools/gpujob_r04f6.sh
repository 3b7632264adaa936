# config E: 128^2 GroupNorms (32 register slots per thread) on the three-kernel path (full-line reads)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04f6; mkdir -p $O
for r in 1 2; do
for T in 32 16; do
for spec in "--size 128 --batch 8 --unet-compute bf16" "--size 64 --batch 8"; do
CFD_GN_BIG_IPT=$T timeout -k 10 200 python tools/kbench.py unet $spec > $O/kb.log 2>&1 || { cat $O/kb.log; exit 5; }
echo "GN_BIG_IPT=$T | $spec | $(grep kernel $O/kb.log | cut -c60-200)"
done; done; done
for T in 32 16; do
CFD_GN_BIG_IPT=$T timeout -k 10 300 python3 tools/kbench.py utrain --batch 16 --size 128 > $O/ut.out 2> $O/ut.err || { tail -20 $O/ut.err; exit 4; }
echo "GN_BIG_IPT=$T $(grep unet_train_step $O/ut.out | cut -c60-220)"
done
