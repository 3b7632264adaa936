# K1h 16-wide halo swizzle: bit-identity against the previous build, timings, bank-conflict PMC
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04z; mkdir -p $O
A=$(CFD_LIB=libconfild_hip_prev.so timeout -k 10 200 python tools/dev/ab_bits.py 2>/dev/null | tail -1) || exit 1
Bh=$(timeout -k 10 200 python tools/dev/ab_bits.py 2>/dev/null | tail -1) || exit 1
echo "prev: $A"; echo "new:  $Bh"; [ "$A" = "$Bh" ] && echo BITIDENTICAL || echo DIFFER
for r in 1 2; do
for L in libconfild_hip_prev.so libconfild_hip.so; do
for spec in "--size 64 --batch 8" "--size 128 --batch 8 --unet-compute bf16"; do
CFD_LIB=$L timeout -k 10 200 python tools/kbench.py unet $spec > $O/kb.log 2>&1 || { cat $O/kb.log; exit 5; }
echo "$L | $spec | $(grep kernel $O/kb.log | cut -c60-200)"
done; done; done
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc -o run -- python3 tools/kbench.py unet --size 64 --batch 8 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 11; }
PMC_ALL=1 python3 tools/convpmc.py $O/pmc 2>&1 | grep conv_h | head
rm -rf $O/pmc
