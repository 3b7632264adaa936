# round 6u: the 8-GPU strong share (one sample per GPU, planned for 1) pipelined at sampling CU
# shares 128..224 (the decode of its 64 rows needs few CUs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06u; mkdir -p $O
PIPE_COUNT=1 PIPE_PLAN=1 timeout -k 10 900 python3 tools/dev/pipe_split.py 128 160 192 224 > $O/pipe_split_b1.jsonl 2> $O/pipe_split_b1.err || { tail -20 $O/pipe_split_b1.err; exit 2; }
cat $O/pipe_split_b1.jsonl
