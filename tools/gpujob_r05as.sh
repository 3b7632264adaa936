# round 5as: interleaved A/B of the conv XCD order (CFD_CONV_XCD 3 vs 1) and the K1s register ring (CFD_CONV_PF 1 vs 2)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05as; mkdir -p $O
i=0
for r in 1 2; do
for e in "X=0" "CFD_CONV_XCD=1" "CFD_CONV_PF=2" "CFD_CONV_XCD=1 CFD_CONV_PF=2"; do
  i=$((i+1))
  env $e LOOP_MODES=2:4 timeout -k 10 300 python3 tools/loop_probe.py E100 B8 B1 A > $O/k$i.out 2> $O/k$i.err || { tail -20 $O/k$i.err; exit 3; }
  python3 -c "
import json
r=[json.loads(l) for l in open('$O/k$i.out') if 'mode' in l]
print('$e', ' '.join('%s=%.3f' % (x['case'], x['ms_per_step']) for x in r))"
done
done
