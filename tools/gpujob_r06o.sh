# round 6o: config B's pipeline at CU splits 96..160 for the sampling stream (the row-split decode
# re-balances itself per batch), two interleaved rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06o; mkdir -p $O
timeout -k 10 900 python3 tools/dev/pipe_split.py 96 112 128 144 160 > $O/pipe_split.jsonl 2> $O/pipe_split.err || { tail -20 $O/pipe_split.err; exit 2; }
cat $O/pipe_split.jsonl
