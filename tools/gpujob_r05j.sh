# round 5j: bf16 qkv-epilogue K/V pack (band-local), K1x bf16 for config E's 8^2 3x3: knob bits (LDSEPI=0
# disables the pack), bf16 + parity suites, then E / B timing with each switched off
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_knobs.py tests/test_gpu_bf16.py tests/test_gpu_parity.py tests/test_gpu_cfg.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for S in "CFD_ATTN_KVFUSE=1" "CFD_ATTN_KVFUSE=0" "CFD_CONV_KXB=0"; do
env $S LOOP_MODES=2:4 timeout -k 10 300 python tools/loop_probe.py B8 E100 > $O/lp.log 2>&1 || { cat $O/lp.log; exit 2; }
echo "$S $(grep -v forward_ms $O/lp.log | grep case | python3 -c 'import sys,json; print(" ".join("%s=%.3f" % (d["case"], d["ms_per_step"]) for d in map(json.loads, sys.stdin)))')"
done; done
