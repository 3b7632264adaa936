# round 5e: K1h 64-channel tiles by plan (CFD_KH_N64 = min per-sample pixels) x skip fusion, graph loop timing
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05e; mkdir -p $O
for r in 1 2; do
for S in "CFD_KH_N64=0" "CFD_KH_N64=4096" "CFD_KH_N64=1024" "CFD_KH_N64=256" "CFD_KH_N64=1024 CFD_CONV_SKIPFUSE=0" "CFD_KH_N64=0 CFD_CONV_SKIPFUSE=0"; do
env $S LOOP_MODES=2:4 timeout -k 10 300 python tools/loop_probe.py A B1 B8 > $O/lp.log 2>&1 || { cat $O/lp.log; exit 2; }
echo "$S $(grep -v forward_ms $O/lp.log | grep case | python3 -c 'import sys,json; print(" ".join("%s=%.3f" % (d["case"], d["ms_per_step"]) for d in map(json.loads, sys.stdin)))')"
done; done
