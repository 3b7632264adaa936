# round 6l: config E re-check (the r06z box ran it 1.65x slower than round 5): the line with one
# warmup step, then the line as the checkpoint ran it, and a kernel trace of the 128^2 bf16 forward
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06l; mkdir -p $O
timeout -k 10 400 python3 bench.py --config E --steps 1 --warmup 1 --no-cpu-baseline > $O/benchE_w1.json 2> $O/benchE_w1.err || { tail -20 $O/benchE_w1.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/benchE_w1.json')); print('E w1', d['value'], d['ms_per_step'], d['roofline_unet']['ms_per_forward'], d['roofline']['launch_ms'])"
timeout -k 10 400 python3 bench.py --config E --steps 1 --warmup 0 --no-cpu-baseline > $O/benchE_w0.json 2> $O/benchE_w0.err || { tail -20 $O/benchE_w0.err; exit 4; }
python3 -c "import json; d=json.load(open('$O/benchE_w0.json')); print('E w0', d['value'], d['ms_per_step'], d['roofline_unet']['ms_per_forward'], d['roofline']['launch_ms'])"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_e -o run -- python3 tools/kbench.py unet --size 128 --batch 8 --bf16 > $O/e.out 2> $O/e.err || { tail -5 $O/e.err; exit 5; }
python3 tools/ktrace.py $O/t_e --per 12 --top 30 > $O/e128b8_ktrace.txt; rm -rf $O/t_e
head -12 $O/e128b8_ktrace.txt
