# round 6v: the 1024-thread GroupNorm with 2 split-K slabs per load round (55 VGPRs: two
# workgroups per CU; the same sums in the same order) -- bit identity, then an interleaved
# A/B of the pipelined config-B step (the sampler on 128 CUs) and the whole-chip graph-loop steps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 600 python3 tools/libdiff.py libconfild_hip.so libconfild_hip_gnun.so > $O/libdiff.json 2> $O/libdiff.err || { cat $O/libdiff.json; tail -20 $O/libdiff.err; exit 1; }
cat $O/libdiff.json
i=0
for r in 1 2; do
for L in libconfild_hip.so libconfild_hip_gnun.so; do
  i=$((i+1))
  CFD_LIB=$L timeout -k 10 400 python3 tools/dev/pipe_split.py 128 > $O/p$i.out 2> $O/p$i.err || { tail -20 $O/p$i.err; exit 2; }
  CFD_LIB=$L LOOP_MODES=2:4 timeout -k 10 300 python3 tools/loop_probe.py B8 B1 A > $O/k$i.out 2> $O/k$i.err || { tail -20 $O/k$i.err; exit 3; }
  python3 -c "
import json
p=[json.loads(l) for l in open('$O/p$i.out')]
r=[json.loads(l) for l in open('$O/k$i.out') if 'mode' in l]
print('$L', 'pipe', ['%.3f' % x['fields_per_s'] for x in p], ' '.join('%s=%.3f' % (x['case'], x['ms_per_step']) for x in r))"
done
done
