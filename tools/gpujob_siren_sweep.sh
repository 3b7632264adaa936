# Same-box sweep of decoder environment settings ($SWEEP): split-decoder GPU tests
# under each setting, then 2 alternating rounds of the decode bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
for V in $SWEEP; do
env $V timeout -k 10 300 python -u -m pytest tests/test_gpu_siren_split.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sw_tests.log 2>&1 || { echo "TESTFAIL $V"; tail -30 gpurun_out/sw_tests.log; exit 1; }
echo "$V $(tail -1 gpurun_out/sw_tests.log)"
done
for r in 1 2; do
for V in $SWEEP; do
env $V timeout -k 10 200 python tools/kbench.py siren --latents 256 > gpurun_out/kb_s.log 2>&1 || { cat gpurun_out/kb_s.log; exit 2; }
echo "$V $(grep -i ms gpurun_out/kb_s.log | tail -1 | cut -c120-220)"
done; done
