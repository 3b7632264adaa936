# attention backward: two interleaved MFMA chains for S and dP
# parity (training, DPS / input-VJP, config-D chains), same-box A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ag; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_unet_train.py tests/test_gpu_dps.py "tests/test_gpu_cfg.py::test_configD_batched_chains_equal_single_chains" "tests/test_gpu_cfg.py::test_configD_dps_steps_at_config_widths" -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for L in libconfild_hip_prev.so libconfild_hip.so; do
CFD_LIB=$L timeout -k 10 300 python3 tools/kbench.py utrain --batch 16 --size 128 > $O/ut.out 2> $O/ut.err || { tail -20 $O/ut.err; exit 4; }
echo "$L $(grep unet_train_step $O/ut.out | cut -c60-300)"
done; done
for L in libconfild_hip_prev.so libconfild_hip.so; do
CFD_LIB=$L timeout -k 10 300 python3 tools/kbench.py dps > $O/dps.out 2> $O/dps.err || { tail -20 $O/dps.err; exit 6; }
echo "$L $(grep -v amdgpu.ids $O/dps.out | tail -1 | cut -c1-300)"
done
