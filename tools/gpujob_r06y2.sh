# round 6 final check y2: the driver's bench command (with its CPU baseline), the default bench
# under a kernel trace, bench lines A / C / D / E / Case4 and the 8-GPU strong share on one GPU
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06y; mkdir -p $O
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/benchB.json 2> $O/benchB.err || { tail -20 $O/benchB.err; exit 3; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 4; }
S=$(find $O/prof_bench -name "*kernel_stats.csv" | head -1); cp $S $O/bench_kernel_stats.csv; rm -rf $O/prof_bench
timeout -k 10 300 python3 bench.py --config A --steps 5 --warmup 1 > $O/benchA.json 2> $O/benchA.err || { tail -20 $O/benchA.err; exit 5; }
timeout -k 10 300 python3 bench.py --config C > $O/benchC.json 2> $O/benchC.err || { tail -20 $O/benchC.err; exit 6; }
timeout -k 10 400 python3 bench.py --config E --steps 1 --warmup 1 > $O/benchE.json 2> $O/benchE.err || { tail -20 $O/benchE.err; exit 7; }
timeout -k 10 300 python3 bench.py --config D --steps 2 --warmup 1 > $O/benchD.json 2> $O/benchD.err || { tail -20 $O/benchD.err; exit 8; }
timeout -k 10 500 python3 bench.py --config Case4 --steps 1 --warmup 1 > $O/benchCase4.json 2> $O/benchCase4.err || { tail -20 $O/benchCase4.err; exit 9; }
timeout -k 10 300 python3 bench.py --per-gpu-batch 1 --steps 8 --warmup 2 --no-cpu-baseline > $O/benchB1.json 2> $O/benchB1.err || { tail -20 $O/benchB1.err; exit 10; }
for c in B A C E D Case4 B1; do python3 -c "import json; d=json.load(open('$O/bench$c.json')); r=d.get('roofline') or {}; print('$c', round(d['value'],3), d['unit'], round(d['ms_per_step'],2), 'ms/step frac', r.get('frac'), 'cpu', d.get('cpu_baseline') and round(d['cpu_baseline']['value'],5))"; done
