# round 5w: planned batch for config A (B = 1) and config B (B = 8): same-box A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05w; mkdir -p $O
for pb in 0 1 2 4 0 2; do
  timeout -k 10 300 python3 bench.py --config A --steps 5 --warmup 1 --no-cpu-baseline --plan-batch $pb > $O/a.json 2> $O/a.err || { tail -20 $O/a.err; exit 3; }
  python3 -c "import json; d=json.load(open('$O/a.json')); print('A pb=$pb', round(d['value'],3), round(d['ms_per_step'],3))"
done
for pb in 0 4 16 0; do
  timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --plan-batch $pb > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 4; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('B pb=$pb', round(d['value'],3), round(d['ms_per_step'],3))"
done
