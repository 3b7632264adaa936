# round 6ac: feasibility of a planner tuned for the sampler's 128-CU half (split-K targets halved,
# development build pc128): interleaved A/B of the pipelined config-B step (128 sampling CUs) and
# of the whole-chip graph-loop step (B = 8)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06ac; mkdir -p $O
i=0
for r in 1 2; do
for L in libconfild_hip.so libconfild_hip_pc128.so; do
  i=$((i+1))
  CFD_LIB=$L timeout -k 10 400 python3 tools/dev/pipe_split.py 128 > $O/p$i.out 2> $O/p$i.err || { tail -20 $O/p$i.err; exit 2; }
  CFD_LIB=$L LOOP_MODES=2:4 timeout -k 10 300 python3 tools/loop_probe.py B8 > $O/k$i.out 2> $O/k$i.err || { tail -20 $O/k$i.err; exit 3; }
  python3 -c "
import json
p=[json.loads(l) for l in open('$O/p$i.out')]
r=[json.loads(l) for l in open('$O/k$i.out') if 'mode' in l]
print('$L', 'pipe', ['%.3f' % x['fields_per_s'] for x in p], [x['rows_b'] for x in p][-1], ' '.join('%s=%.3f' % (x['case'], x['ms_per_step']) for x in r))"
done
done
