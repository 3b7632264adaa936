# round 6q: key-chunked split attention (kc > 1 where the planned batch's grid is small): parity
# (forward goldens, plan invariance, DPS VJP, the 256-step loop at plans 1 / 2, knobs), then an
# interleaved A/B against the no-chunk build of the graph-loop step at plan 8 (E100, B8, B1, A)
# and plan 1 (B1, A)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06q; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_plan_batch.py tests/test_gpu_dps.py "tests/test_gpu_cfg.py::test_configB_full_256_step_trajectory" "tests/test_gpu_cfg.py::test_configA_ddim50_and_decode_end_to_end" tests/test_gpu_knobs.py tests/test_gpu_unet_train.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 5; }
tail -1 $O/tests.log
i=0
for r in 1 2; do
for L in libconfild_hip_nokc.so libconfild_hip.so; do
  i=$((i+1))
  CFD_LIB=$L LOOP_MODES=2:4 timeout -k 10 300 python3 tools/loop_probe.py E100 B8 B1 A > $O/k$i.out 2> $O/k$i.err || { tail -20 $O/k$i.err; exit 3; }
  CFD_LIB=$L LOOP_PLAN=1 LOOP_MODES=2:4 timeout -k 10 300 python3 tools/loop_probe.py B1 A > $O/p$i.out 2> $O/p$i.err || { tail -20 $O/p$i.err; exit 4; }
  python3 -c "
import json
r=[json.loads(l) for l in open('$O/k$i.out') if 'mode' in l]
p=[json.loads(l) for l in open('$O/p$i.out') if 'mode' in l]
print('$L', ' '.join('%s=%.3f' % (x['case'], x['ms_per_step']) for x in r), '| plan1', ' '.join('%s=%.3f' % (x['case'], x['ms_per_step']) for x in p))"
done
done
