# round 6w: no split-K for the transposed 1x1 convolutions with >= 128 tiles (as the forward's):
# DPS parity on the variant build, then an interleaved A/B of the config-D DPS step and its parts
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06w; mkdir -p $O
CFD_LIB=libconfild_hip_t1x1.so timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_dps.py "tests/test_gpu_cfg.py::test_configD_dps_steps_at_config_widths" "tests/test_gpu_cfg.py::test_configD_batched_chains_equal_single_chains" "tests/test_gpu_cfg.py::test_configD_dps_chain_vs_oracle" > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 5; }
tail -1 $O/tests.log
i=0
for r in 1 2 3; do
for L in libconfild_hip.so libconfild_hip_t1x1.so; do
  i=$((i+1))
  CFD_LIB=$L timeout -k 10 300 python3 tools/kbench.py dps --batch 8 > $O/d$i.out 2> $O/d$i.err || { tail -20 $O/d$i.err; exit 4; }
  python3 -c "
import json
d=json.loads(open('$O/d$i.out').read().strip().splitlines()[-1])
print('$L', 'dps_step=%.3f vjp=%.3f fwdtape=%.3f' % (d['step_ms'], d['unet_vjp_ms'], d['unet_fwd_tape_ms']))"
done
done
