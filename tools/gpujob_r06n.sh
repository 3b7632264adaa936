# round 6n: small-batch U-Net forwards at planned batch 8 / 1 / 2 (config A's 32^2 and the
# strong share's 64^2 at B = 1), and kernel traces of both at plan 1
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06n; mkdir -p $O
for p in 0 1 2; do
  timeout -k 10 200 python3 tools/kbench.py unet --size 32 --mult 1,2,3,4 --batch 1 --plan $p >> $O/kbench.jsonl 2>> $O/kbench.err || { tail -5 $O/kbench.err; exit 2; }
  timeout -k 10 200 python3 tools/kbench.py unet --size 64 --batch 1 --plan $p >> $O/kbench.jsonl 2>> $O/kbench.err || { tail -5 $O/kbench.err; exit 3; }
done
cat $O/kbench.jsonl
run_trace() {  # name, per, command...
  n=$1; per=$2; shift 2
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_$n -o run -- "$@" > $O/$n.out 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  S=$(find $O/t_$n -name "*kernel_stats.csv" | head -1); cp $S $O/${n}_kernel_stats.csv
  python3 tools/ktrace.py $O/t_$n --per $per --top 40 > $O/${n}_ktrace.txt
  rm -rf $O/t_$n
  head -22 $O/${n}_ktrace.txt
}
run_trace b64b1p1 12 python3 tools/kbench.py unet --size 64 --batch 1 --plan 1 || exit 4
run_trace a32b1p1 12 python3 tools/kbench.py unet --size 32 --mult 1,2,3,4 --batch 1 --plan 1 || exit 5
