# round 6p: config E's whole 1000-step loop against the reference's run (split-f16 and bf16:
# measures the bf16 drift), then config B's pipeline at CU splits 96..160
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06p; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread "tests/test_gpu_cfg.py::test_configE_full_1000_step_loop" > $O/tests.log 2>&1; rc=$?
grep -E "config E|passed|failed|Error" $O/tests.log | head -10
[ $rc -le 1 ] || exit 5
timeout -k 10 900 python3 tools/dev/pipe_split.py 96 112 128 144 160 > $O/pipe_split.jsonl 2> $O/pipe_split.err || { tail -20 $O/pipe_split.err; exit 2; }
cat $O/pipe_split.jsonl
