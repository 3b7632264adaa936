# round 6b: the switch cleanup -- bit identity of the new library against the pre-cleanup
# build over forwards / input-VJPs / parameter gradients / decodes, then the whole GPU suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 600 python3 tools/libdiff.py libconfild_hip_pre.so libconfild_hip.so > $O/libdiff.json 2> $O/libdiff.err || { cat $O/libdiff.json; tail -20 $O/libdiff.err; exit 1; }
cat $O/libdiff.json
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error" $O/gpu_tests.log | head; tail -30 $O/gpu_tests.log; exit 2; }
tail -1 $O/gpu_tests.log
