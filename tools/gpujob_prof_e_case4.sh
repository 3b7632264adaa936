# config E bf16 U-Net kernel trace (+conv plan log), Case4 DPS kernel stats, bench lines A / E / D / Case4 with CPU baselines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pe; mkdir -p $O
CFD_CONV_LOG=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e -o run -- python3 tools/kbench.py unet --size 128 --batch 8 --bf16 > $O/e128.out 2> $O/e128.err || { tail -20 $O/e128.err; exit 3; }
T=$(find $O/prof_e -name "*kernel_trace.csv" | head -1); cp $T $O/e128_trace.csv
S=$(find $O/prof_e -name "*kernel_stats.csv" | head -1); cp $S $O/e128_stats.csv; rm -rf $O/prof_e
cat $O/e128.out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 bench.py --config Case4 --dps-steps 20 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4prof.out 2> $O/c4prof.err || { tail -20 $O/c4prof.err; exit 4; }
S=$(find $O/prof_c4 -name "*kernel_stats.csv" | head -1); cp $S $O/case4_stats.csv; rm -rf $O/prof_c4
timeout -k 10 300 python3 bench.py --config A --steps 5 --warmup 1 > $O/benchA.json 2> $O/benchA.err || { tail -20 $O/benchA.err; exit 5; }
timeout -k 10 400 python3 bench.py --config E --steps 1 --warmup 0 > $O/benchE.json 2> $O/benchE.err || { tail -20 $O/benchE.err; exit 6; }
timeout -k 10 300 python3 bench.py --config D --steps 2 --warmup 1 > $O/benchD.json 2> $O/benchD.err || { tail -20 $O/benchD.err; exit 7; }
timeout -k 10 400 python3 bench.py --config Case4 --steps 1 --warmup 1 > $O/benchCase4.json 2> $O/benchCase4.err || { tail -20 $O/benchCase4.err; exit 8; }
for c in A E D Case4; do python3 -c "import json; d=json.load(open('$O/bench$c.json')); print('$c', round(d['value'],3), d['unit'], round(d['ms_per_step'],2), 'ms/step', 'cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value'],5))"; done
