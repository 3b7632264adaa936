# round 5aj: config E GroupNorm reach (gn2 from 4096 / 1024 / 256 pixels) and planned batch 16, graph-loop ms per step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05aj; mkdir -p $O
for r in 1 2; do
for S in "CFD_GN2_HW=4096" "CFD_GN2_HW=1024" "CFD_GN2_HW=256" "CFD_PLAN_B=16"; do
env $S LOOP_MODES=2:4 timeout -k 10 300 python tools/loop_probe.py E100 > $O/lp.log 2>&1 || { cat $O/lp.log; exit 2; }
echo "$S $(grep -v forward_ms $O/lp.log | grep case | python3 -c 'import sys,json; print(" ".join("%s=%.3f" % (d["case"], d["ms_per_step"]) for d in map(json.loads, sys.stdin)))')"
done; done
