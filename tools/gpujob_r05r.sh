# round 5r: does the per-model plan batch reach the planner (Case4 conv log, env vs handle)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05r; mkdir -p $O
CFD_CONV_LOG=1 timeout -k 10 200 python3 bench.py --config Case4 --dps-steps 1 --steps 1 --warmup 0 --no-cpu-baseline > $O/h.out 2> $O/h.err || { tail -20 $O/h.err; exit 3; }
CFD_PLAN_B=2 CFD_CONV_LOG=1 timeout -k 10 200 python3 bench.py --config Case4 --dps-steps 1 --steps 1 --warmup 0 --no-cpu-baseline > $O/e.out 2> $O/e.err || { tail -20 $O/e.err; exit 4; }
grep CONV $O/h.err | head -30
diff <(grep CONV $O/h.err) <(grep CONV $O/e.err) | head -20
for e in "X=0" "CFD_PLAN_B=2" "X=0" "CFD_PLAN_B=2"; do
  env $e timeout -k 10 200 python3 bench.py --config Case4 --dps-steps 30 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4ab.json 2> $O/c4ab.err || { tail -20 $O/c4ab.err; exit 8; }
  python3 -c "import json; d=json.load(open('$O/c4ab.json')); print('$e', round(d['value'],3), round(d['ms_per_step'],3))"
done
