# round 5q: planner nominal batch per model (Case4: 2) + K1s at the large latents; GN backward A/B at config D
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_plan_batch.py tests/test_gpu_dps.py tests/test_gpu_cfg.py -k "plan or dps or vjp or configD or case4" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
for e in "X=0" "CFD_GNB2=0" "X=0" "CFD_GNB2=0"; do
  env $e timeout -k 10 200 python3 tools/kbench.py dps --batch 8 > $O/d.out 2> $O/d.err || { tail -20 $O/d.err; exit 5; }
  echo "$e $(python3 -c "import json; d=json.load(open('$O/d.out')); print(round(d['step_ms'],3), round(d['unet_vjp_ms'],3))")"
done
for e in "X=0" "CFD_CONV_K1S_HW=0" "X=0"; do
  env $e timeout -k 10 200 python3 bench.py --config Case4 --dps-steps 30 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4ab.json 2> $O/c4ab.err || { tail -20 $O/c4ab.err; exit 8; }
  python3 -c "import json; d=json.load(open('$O/c4ab.json')); print('$e', round(d['value'],3), round(d['ms_per_step'],3))"
done
