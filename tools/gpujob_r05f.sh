# round 5f: two-launch full-row GroupNorm (CFD_GN2_HW) parity + timing sweep; conv_in/out grid-stride
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05f; mkdir -p $O
CFD_GN2_HW=1024 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_unet_split.py tests/test_gpu_bf16.py -x -q --timeout 300 --timeout-method thread > $O/tests_gn2.log 2>&1 || { tail -40 $O/tests_gn2.log; exit 1; }
tail -1 $O/tests_gn2.log
for r in 1 2; do
for S in "CFD_GN2_HW=0" "CFD_GN2_HW=16384" "CFD_GN2_HW=4096" "CFD_GN2_HW=1024"; do
env $S LOOP_MODES=2:4 timeout -k 10 300 python tools/loop_probe.py A B1 B8 E100 > $O/lp.log 2>&1 || { cat $O/lp.log; exit 2; }
echo "$S $(grep -v forward_ms $O/lp.log | grep case | python3 -c 'import sys,json; print(" ".join("%s=%.3f" % (d["case"], d["ms_per_step"]) for d in map(json.loads, sys.stdin)))')"
done; done
