# round 6i: (1) [removed: the 512-thread GroupNorm tier measured flat]; (2) parity subset + the pipeline tests (row-split
# decode); (3) the driver's bench command with the row-split pipeline; (4) DPS kernel traces
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06i; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_plan_batch.py tests/test_gpu_unet_split.py "tests/test_gpu_cfg.py::test_configB_full_256_step_trajectory" "tests/test_gpu_cfg.py::test_configA_ddim50_and_decode_end_to_end" tests/test_gpu_dps.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 5; }
tail -1 $O/tests.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 6; }
python3 -c "import json; d=json.load(open('$O/bench.json')); p=d['pipeline']; print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['frac_chip'], p['sample_ms_per_batch'], p['decode_half_ms_per_batch'], p['decode_half_rows'])"
run_trace() {  # name, per, command...
  n=$1; per=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_$n -o run -- "$@" > $O/$n.out 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  S=$(find $O/t_$n -name "*kernel_stats.csv" | head -1); cp $S $O/${n}_kernel_stats.csv
  python3 tools/ktrace.py $O/t_$n --per $per --top 30 > $O/${n}_ktrace.txt
  rm -rf $O/t_$n
  head -14 $O/${n}_ktrace.txt
}
run_trace dpsD 20 python3 bench.py --config D --steps 1 --warmup 0 --dps-steps 20 --no-cpu-baseline || exit 7
run_trace dpsCase4 20 python3 bench.py --config Case4 --steps 1 --warmup 0 --dps-steps 20 --no-cpu-baseline || exit 8
