# Same-box A/B of the decoder under two environment settings (AB_A / AB_B): the
# split-decoder GPU tests under AB_B, then 3 alternating rounds of the decode bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
env $AB_B timeout -k 10 400 python -u -m pytest tests/test_gpu_siren_split.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for r in 1 2 3; do
for V in "$AB_A" "$AB_B"; do
env $V timeout -k 10 200 python tools/kbench.py siren --latents 256 > gpurun_out/kb_s.log 2>&1 || { cat gpurun_out/kb_s.log; exit 2; }
echo "$V $(grep -i ms gpurun_out/kb_s.log | tail -1 | cut -c1-220)"
done; done
