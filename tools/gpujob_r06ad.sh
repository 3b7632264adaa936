# round 6ad: the pipelined config-B step (128 sampling CUs) under the bit-identical schedule
# switches (XCD orders of the convolution tiles and of the attention workgroups), two rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06ad; mkdir -p $O
for r in 1 2; do
for cfg in "X=0" "CFD_ATTN_XCD=0" "CFD_CONV_XCD=1" "CFD_CONV_XCD=2" "CFD_CONV_XCD=0"; do
  env $cfg timeout -k 10 400 python3 tools/dev/pipe_split.py 128 > $O/p.out 2> $O/p.err || { tail -20 $O/p.err; exit 2; }
  python3 -c "
import json
p=[json.loads(l) for l in open('$O/p.out')]
print('$cfg', ['%.3f' % x['fields_per_s'] for x in p])"
done
done
