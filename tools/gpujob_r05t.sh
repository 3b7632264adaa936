# round 5t: real Case4 kernel trace at HEAD (plan batch 2, K1s at the large latents)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 bench.py --config Case4 --dps-steps 20 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4.out 2> $O/c4.err || { tail -20 $O/c4.err; exit 4; }
cat $O/c4.out
S=$(find $O/prof_c4 -name "*kernel_stats.csv" | head -1); cp $S $O/c4_stats.csv
T=$(find $O/prof_c4 -name "*kernel_trace.csv" | head -1); gzip -c $T > $O/c4_trace.csv.gz; rm -rf $O/prof_c4
