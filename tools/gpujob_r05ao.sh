# round 5ao: config E (bf16 128^2, B = 8) kernel stats at HEAD (native graph loop, 100 steps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ao; mkdir -p $O
LOOP_MODES=2:4 timeout -k 10 300 python3 tools/loop_probe.py E100 > $O/e.out 2> $O/e.err || { tail -20 $O/e.err; exit 3; }
cat $O/e.out
LOOP_MODES=2:4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/loop_probe.py E100 > $O/ep.out 2> $O/ep.err || { tail -20 $O/ep.err; exit 4; }
S=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $S $O/e_stats.csv
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); gzip -c $T > $O/e_trace.csv.gz; rm -rf $O/prof
