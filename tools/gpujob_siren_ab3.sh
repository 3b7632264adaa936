# Same-box A/B/C of the decoder under three environment settings (AB_A, AB_B, AB_C):
# the split-decoder GPU tests under the default, then 3 alternating rounds of the
# config-B decode bench (256 latents).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_siren_split.py tests/test_gpu_parity.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo TESTFAIL; grep -E "sine|err|FAIL|Error" gpurun_out/ab_tests.log | tail -30; exit 1; }
grep -E "sine|max err" gpurun_out/ab_tests.log | cut -c1-200
tail -1 gpurun_out/ab_tests.log
for r in 1 2 3; do
for V in "$AB_A" "$AB_B" "$AB_C"; do
env $V timeout -k 10 200 python tools/kbench.py siren --latents 256 > gpurun_out/kb_s.log 2>&1 || { cat gpurun_out/kb_s.log; exit 2; }
echo "$V $(grep -i ms gpurun_out/kb_s.log | tail -1 | cut -c1-220)"
done; done
