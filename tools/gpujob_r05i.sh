# round 5i: K1hb three taps per step (bf16, config E): bf16 parity + knob bits, then E / B timing, KHB_OCC A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05i; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_knobs.py -x -q --timeout 300 --timeout-method thread -k "bf16 or KHB or schedule" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for S in "CFD_CONV_KHB_OCC=1" "CFD_CONV_KHB_OCC=0"; do
env $S LOOP_MODES=2:4 timeout -k 10 300 python tools/loop_probe.py E100 > $O/lp.log 2>&1 || { cat $O/lp.log; exit 2; }
echo "$S $(grep -v forward_ms $O/lp.log | grep case | python3 -c 'import sys,json; print(" ".join("%s=%.3f" % (d["case"], d["ms_per_step"]) for d in map(json.loads, sys.stdin)))')"
done; done
