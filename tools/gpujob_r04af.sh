# parity after the GroupNorm range / bounded gn_apply changes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04af; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_unet_train.py tests/test_gpu_dps.py tests/test_gpu_cfg.py tests/test_gpu_knobs.py -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
