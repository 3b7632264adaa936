# round 5ap: K1s split-K target (CFD_CONV_TARGET_WG) sweep -- config E (bf16 128^2 B = 8), B = 8 64^2, config A
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ap; mkdir -p $O
for t in 768 384 512 1024 256 768; do
  CFD_CONV_TARGET_WG=$t LOOP_MODES=2:4 timeout -k 10 300 python3 tools/loop_probe.py E100 B8 A > $O/t$t.out 2> $O/t$t.err || { tail -20 $O/t$t.err; exit 3; }
  python3 -c "
import json
r=[json.loads(l) for l in open('$O/t$t.out') if 'mode' in l]
print('TARGET_WG=$t', ' '.join('%s=%.3f' % (x['case'], x['ms_per_step']) for x in r))"
done
