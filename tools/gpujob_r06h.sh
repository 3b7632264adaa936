# round 6h: 512-thread GroupNorm tier (the 32^2 level) A/B against the 256-tier build; parity subset;
# kernel traces of 20 guided steps at config D (8 chains) and real Case4 (one chain)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06h; mkdir -p $O
i=0
for r in 1 2 3; do
for L in libconfild_hip_exp2.so libconfild_hip_exp3.so; do
  i=$((i+1))
  CFD_LIB=$L LOOP_MODES=2:4 timeout -k 10 300 python3 tools/loop_probe.py E100 B8 B1 A > $O/k$i.out 2> $O/k$i.err || { tail -20 $O/k$i.err; exit 3; }
  python3 -c "
import json
r=[json.loads(l) for l in open('$O/k$i.out') if 'mode' in l]
print('$L', ' '.join('%s=%.3f' % (x['case'], x['ms_per_step']) for x in r))"
done
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_plan_batch.py tests/test_gpu_unet_split.py "tests/test_gpu_cfg.py::test_configB_full_256_step_trajectory" "tests/test_gpu_cfg.py::test_configA_ddim50_and_decode_end_to_end" tests/test_gpu_dps.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 5; }
tail -1 $O/tests.log
run_trace() {  # name, per, command...
  n=$1; per=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_$n -o run -- "$@" > $O/$n.out 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  S=$(find $O/t_$n -name "*kernel_stats.csv" | head -1); cp $S $O/${n}_kernel_stats.csv
  python3 tools/ktrace.py $O/t_$n --per $per --top 30 > $O/${n}_ktrace.txt
  rm -rf $O/t_$n
  head -14 $O/${n}_ktrace.txt
}
run_trace dpsD 20 python3 bench.py --config D --steps 1 --warmup 0 --dps-steps 20 --no-cpu-baseline || exit 6
run_trace dpsCase4 20 python3 bench.py --config Case4 --steps 1 --warmup 0 --dps-steps 20 --no-cpu-baseline || exit 7
