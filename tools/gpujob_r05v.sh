# round 5v: GroupNorm chunking by planned batch: parity + config D / Case4
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_plan_batch.py tests/test_gpu_dps.py tests/test_gpu_cfg.py tests/test_gpu_unet_split.py -k "plan or dps or vjp or configD or case4 or split" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
for e in "X=0" "CFD_GNB2=2" "X=0"; do
  env $e timeout -k 10 200 python3 tools/kbench.py dps --batch 8 > $O/d.out 2> $O/d.err || { tail -20 $O/d.err; exit 5; }
  echo "$e $(python3 -c "import json; d=json.load(open('$O/d.out')); print(round(d['step_ms'],3), round(d['unet_vjp_ms'],3))")"
done
for pb in 2 1 0 2 1; do
  timeout -k 10 200 python3 bench.py --config Case4 --dps-steps 30 --steps 1 --warmup 1 --no-cpu-baseline --plan-batch $pb > $O/c4ab.json 2> $O/c4ab.err || { tail -20 $O/c4ab.err; exit 8; }
  python3 -c "import json; d=json.load(open('$O/c4ab.json')); print('pb=$pb', round(d['value'],3), round(d['ms_per_step'],3))"
done
