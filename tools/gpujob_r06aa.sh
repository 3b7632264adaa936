# round 6aa: real Case4 DPS (one chain) at planned batch 1 / 2 / 4 (the line runs at 2)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06aa; mkdir -p $O
for r in 1 2; do
for p in 1 2 4; do
  timeout -k 10 500 python3 bench.py --config Case4 --steps 1 --warmup 1 --no-cpu-baseline --plan-batch $p > $O/c4_p${p}_r$r.json 2> $O/c4_p${p}_r$r.err || { tail -20 $O/c4_p${p}_r$r.err; exit 2; }
  python3 -c "import json; d=json.load(open('$O/c4_p${p}_r$r.json')); print('plan $p', d['value'], d['ms_per_step'])"
done
done
