# K1x with two K tiles in flight at the small levels (CFD_CONVX_PF=2): bit-identity, timings
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04f5; mkdir -p $O
A=$(timeout -k 10 200 python tools/dev/ab_bits.py 2>/dev/null | tail -1) || exit 1
B=$(CFD_CONVX_PF=2 timeout -k 10 200 python tools/dev/ab_bits.py 2>/dev/null | tail -1) || exit 1
echo "pf1: $A"; echo "pf2: $B"; [ "$A" = "$B" ] && echo BITIDENTICAL || echo DIFFER
for r in 1 2; do
for P in 1 2; do
for spec in "--size 64 --batch 8" "--size 64 --batch 1" "--size 32 --mult 1,2,3,4 --batch 1"; do
CFD_CONVX_PF=$P timeout -k 10 200 python tools/kbench.py unet $spec > $O/kb.log 2>&1 || { cat $O/kb.log; exit 5; }
echo "CONVX_PF=$P | $spec | $(grep kernel $O/kb.log | cut -c60-200)"
done; done; done
