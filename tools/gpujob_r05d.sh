# round 5d: fused skip convolution (K1h XF) parity + A/B CFD_CONV_SKIPFUSE 0 / 1 / 2 (graph loop)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_gpu_knobs.py tests/test_gpu_native_loop.py tests/test_gpu_dps.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/dev/env_bits.py "CFD_CONV_SKIPFUSE=0" "" "CFD_CONV_SKIPFUSE=2" || exit 3
rm -rf gpurun_out/envbits
for r in 1 2; do
for S in 0 1 2; do
CFD_CONV_SKIPFUSE=$S LOOP_MODES=2:4 timeout -k 10 300 python tools/loop_probe.py A B1 B8 > $O/lp.log 2>&1 || { cat $O/lp.log; exit 2; }
echo "SKIPFUSE=$S"; grep -v forward_ms $O/lp.log | cut -c1-130
done; done
