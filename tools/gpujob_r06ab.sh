# round 6ab: K9t forward timing experiments (development builds, wrong results by design):
# 1 = no sine in the epilogue, 2 = no per-block barrier, 3 = no wait for the weight DMA
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06ab; mkdir -p $O
timeout -k 10 600 python3 tools/dev/tape_bench.py libconfild_hip.so libconfild_hip_k9e1.so libconfild_hip_k9e2.so libconfild_hip_k9e3.so > $O/tape_exp.json 2> $O/tape_exp.err || { tail -20 $O/tape_exp.err; exit 2; }
python3 -c "
import json; d=json.load(open('$O/tape_exp.json'))
for lib, rows in d.items():
    for r in rows: print(lib, {k: (round(v['fwd_ms'],3), round(v['vjp_ms'],3)) for k, v in r.items()})"
