# round 5ar: knob sweep at HEAD -- gn2 reach (CFD_GN2_HW), conv XCD order, K1s register ring -- config E / B = 8 / config A
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ar; mkdir -p $O
i=0
for e in "X=0" "CFD_GN2_HW=1024" "CFD_GN2_HW=256" "CFD_CONV_XCD=1" "CFD_CONV_PF=2" "X=0"; do
  i=$((i+1))
  env $e LOOP_MODES=2:4 timeout -k 10 300 python3 tools/loop_probe.py E100 B8 A > $O/k$i.out 2> $O/k$i.err || { tail -20 $O/k$i.err; exit 3; }
  python3 -c "
import json
r=[json.loads(l) for l in open('$O/k$i.out') if 'mode' in l]
print('$e', ' '.join('%s=%.3f' % (x['case'], x['ms_per_step']) for x in r))"
done
