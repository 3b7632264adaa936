# round 6j: K9t (split-f16 DPS tape kernels): DPS / CNF-training parity, then kernel traces of
# config D and real Case4 DPS steps at ring depth 2 and 3, and the config-D / Case4 bench lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_dps.py tests/test_gpu_cnftrain.py tests/test_gpu_cfg.py -k "dps or tape or configD or case4 or train" > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 5; }
tail -1 $O/tests.log
run_trace() {  # name, per, command...
  n=$1; per=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_$n -o run -- "$@" > $O/$n.out 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  S=$(find $O/t_$n -name "*kernel_stats.csv" | head -1); cp $S $O/${n}_kernel_stats.csv
  python3 tools/ktrace.py $O/t_$n --per $per --top 30 > $O/${n}_ktrace.txt
  rm -rf $O/t_$n
  grep -E "total|siren_tape" $O/${n}_ktrace.txt
}
run_trace dpsD_r2 20 python3 bench.py --config D --steps 1 --warmup 0 --dps-steps 20 --no-cpu-baseline || exit 7
CFD_TAPE_RING=3 run_trace dpsD_r3 20 python3 bench.py --config D --steps 1 --warmup 0 --dps-steps 20 --no-cpu-baseline || exit 8
run_trace dpsCase4_r2 20 python3 bench.py --config Case4 --steps 1 --warmup 0 --dps-steps 20 --no-cpu-baseline || exit 9
CFD_TAPE_RING=3 run_trace dpsCase4_r3 20 python3 bench.py --config Case4 --steps 1 --warmup 0 --dps-steps 20 --no-cpu-baseline || exit 10
for r in 2 3; do
  CFD_TAPE_RING=$r timeout -k 10 300 python3 bench.py --config D --steps 2 --warmup 1 --no-cpu-baseline > $O/benchD_r$r.json 2> $O/benchD_r$r.err || { tail -20 $O/benchD_r$r.err; exit 11; }
  python3 -c "import json; d=json.load(open('$O/benchD_r$r.json')); print('D ring $r', d['value'], d['ms_per_step'])"
done
