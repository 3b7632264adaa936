# round 6g: 256-thread GroupNorm workgroups for the small groups (16^2 / 8^2 levels): interleaved
# A/B of the graph-loop step against the previous build, then the parity suites that run them
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06g; mkdir -p $O
i=0
for r in 1 2 3; do
for L in libconfild_hip_exp.so libconfild_hip_exp2.so; do
  i=$((i+1))
  CFD_LIB=$L LOOP_MODES=2:4 timeout -k 10 300 python3 tools/loop_probe.py E100 B8 B1 A > $O/k$i.out 2> $O/k$i.err || { tail -20 $O/k$i.err; exit 3; }
  python3 -c "
import json
r=[json.loads(l) for l in open('$O/k$i.out') if 'mode' in l]
print('$L', ' '.join('%s=%.3f' % (x['case'], x['ms_per_step']) for x in r))"
done
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_plan_batch.py tests/test_gpu_unet_split.py tests/test_gpu_bf16.py "tests/test_gpu_cfg.py::test_configB_full_256_step_trajectory" "tests/test_gpu_cfg.py::test_configA_ddim50_and_decode_end_to_end" tests/test_gpu_dps.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 5; }
tail -2 $O/tests.log
