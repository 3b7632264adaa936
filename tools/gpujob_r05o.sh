# round 5o: Case4 (one chain) under nominal plan batches 1 / 2 / 4 and K1s-only variants
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05o; mkdir -p $O
for e in "X=0" "CFD_PLAN_B=1" "CFD_PLAN_B=2" "CFD_PLAN_B=4" "CFD_PLAN_B=1 CFD_CONV_KX=0" "CFD_PLAN_B=1 CFD_CONV_KH=0" "CFD_PLAN_B=1 CFD_GNB2=0" "X=0"; do
  env $e timeout -k 10 200 python3 bench.py --config Case4 --dps-steps 30 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4ab.json 2> $O/c4ab.err || { tail -20 $O/c4ab.err; exit 8; }
  python3 -c "import json; d=json.load(open('$O/c4ab.json')); print('$e', round(d['value'],3), round(d['ms_per_step'],3))"
done
