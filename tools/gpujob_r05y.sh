# round 5y: B = 1 64^2 / config A / B = 8 graph-loop step under planned batches 8 / 1 / 2 / 4
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05y; mkdir -p $O
for r in 1 2; do
for S in "CFD_PLAN_B=8" "CFD_PLAN_B=1" "CFD_PLAN_B=2" "CFD_PLAN_B=4"; do
env $S LOOP_MODES=2:4 timeout -k 10 300 python tools/loop_probe.py B1 A > $O/lp.log 2>&1 || { cat $O/lp.log; exit 2; }
echo "$S $(grep -v forward_ms $O/lp.log | grep case | python3 -c 'import sys,json; print(" ".join("%s=%.3f" % (d["case"], d["ms_per_step"]) for d in map(json.loads, sys.stdin)))')"
done; done
