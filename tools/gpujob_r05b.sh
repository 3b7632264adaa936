# round 5b: side-stream skip convolutions / temb MLP and the qkv-epilogue K/V pack: parity + native-loop
# graphs, then A/B of CFD_UNET_SIDE and CFD_ATTN_KVFUSE (loop_probe, graph mode, unroll 4)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_native_loop.py tests/test_gpu_knobs.py tests/test_gpu_dps.py tests/test_gpu_unet_split.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
for S in "CFD_UNET_SIDE=0 CFD_ATTN_KVFUSE=0" "CFD_UNET_SIDE=1 CFD_ATTN_KVFUSE=0" "CFD_UNET_SIDE=1 CFD_ATTN_KVFUSE=1"; do
env $S LOOP_MODES=2:4 timeout -k 10 300 python tools/loop_probe.py A B1 B8 > $O/lp.log 2>&1 || { cat $O/lp.log; exit 2; }
echo "$S"; grep -v forward_ms $O/lp.log | cut -c1-150
done; done
