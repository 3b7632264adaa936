# attention workgroups grouped per XCD: bit-identity (knob test), timings, L2 hit rate
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04aa; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_knobs.py -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for X in 0 1; do
for spec in "--size 64 --batch 8" "--size 128 --batch 8 --unet-compute bf16" "--size 64 --batch 1"; do
CFD_ATTN_XCD=$X timeout -k 10 200 python tools/kbench.py unet $spec > $O/kb.log 2>&1 || { cat $O/kb.log; exit 5; }
echo "ATTN_XCD=$X | $spec | $(grep kernel $O/kb.log | cut -c60-200)"
done; done; done
for X in 0 1; do
CFD_ATTN_XCD=$X timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc$X -o run -- python3 tools/kbench.py unet --size 64 --batch 8 > $O/pmc$X.log 2>&1 || { tail -5 $O/pmc$X.log; exit 11; }
echo "ATTN_XCD=$X"; PMC_ALL=1 python3 tools/convpmc.py $O/pmc$X 2>&1 | grep attention
rm -rf $O/pmc$X
done
