# round 6a: the new timed-configuration parity tests (PipelineB vs step_B, RCCL gather on the
# CU-masked stream, config-B 256 steps at plans 8/1/2, real Case4 chain at plan 2) and the
# per-tape layout registry; then the plan-batch / DPS suites they touch
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06a; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_pipeline.py tests/test_gpu_unet_train.py tests/test_gpu_plan_batch.py \
  "tests/test_gpu_cfg.py::test_configB_full_256_step_trajectory" \
  "tests/test_gpu_cfg.py::test_case4_real_shape_10_consecutive_dps_steps" \
  tests/test_gpu_dps.py tests/test_gpu_streams.py -s > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head -20; tail -40 $O/tests.log; exit 1; }
grep -E "PASS|drift|chain at plan" $O/tests.log | tail -40
tail -2 $O/tests.log
