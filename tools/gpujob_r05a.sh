# round 5a: tape-mode / split-wgrad tests, XCD tile order A/B (CFD_CONV_XCD 1 vs 3), 16^2 K1h L2 PMC with order 3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet_train.py tests/test_gpu_dps.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
for X in 1 3; do
for spec in "--size 64 --batch 8" "--size 64 --batch 1" "--size 32 --mult 1,2,3,4 --batch 1"; do
CFD_CONV_XCD=$X timeout -k 10 120 python tools/kbench.py unet $spec > $O/kb.log 2>&1 || { cat $O/kb.log; exit 2; }
echo "XCD=$X $spec $(grep kernel $O/kb.log | cut -c1-200)"
done; done; done
i=0
for P in "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" "FETCH_SIZE"; do
  i=$((i+1))
  CFD_CONV_XCD=3 timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/upmc$i -o run -- python3 tools/kbench.py unet --size 64 --batch 8 > $O/upmc$i.log 2>&1 || { tail -5 $O/upmc$i.log; exit 11; }
done
PMC_ALL=1 python3 tools/convpmc.py $O/upmc1 $O/upmc2 > $O/xcd3_unet_pmc.txt 2>&1 || true
rm -rf $O/upmc1 $O/upmc2
grep conv_h $O/xcd3_unet_pmc.txt
