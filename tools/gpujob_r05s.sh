# round 5s: Case4 one chain, same box: planner nominal batch x K1s rule
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05s; mkdir -p $O
for rep in 1 2; do
for e in "0 X=0" "0 CFD_CONV_K1S_HW=0" "2 CFD_CONV_K1S_HW=0" "2 X=0" "1 X=0" "4 X=0"; do
  set -- $e; pb=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --config Case4 --dps-steps 30 --steps 1 --warmup 1 --no-cpu-baseline --plan-batch $pb > $O/c4ab.json 2> $O/c4ab.err || { tail -20 $O/c4ab.err; exit 8; }
  python3 -c "import json; d=json.load(open('$O/c4ab.json')); print('pb=$pb $*', round(d['value'],3), round(d['ms_per_step'],3))"
done
done
