# round 5au: DPS knob sweep -- config D step (kbench) and real Case4 (30 steps, one chain) under conv schedule knobs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05au; mkdir -p $O
i=0
for e in "X=0" "CFD_CONV_XCD=1" "CFD_CONV_TARGET_WG=384" "CFD_CONV_TARGET_WG=1536" "CFD_CONV_KMIN=2" "X=0"; do
  i=$((i+1))
  env $e timeout -k 10 200 python3 tools/kbench.py dps --batch 8 > $O/d$i.out 2> $O/d$i.err || { tail -20 $O/d$i.err; exit 5; }
  env $e timeout -k 10 200 python3 bench.py --config Case4 --dps-steps 30 --steps 1 --warmup 1 --no-cpu-baseline > $O/c$i.json 2> $O/c$i.err || { tail -20 $O/c$i.err; exit 8; }
  python3 -c "
import json; d=json.load(open('$O/d$i.out')); c=json.load(open('$O/c$i.json'))
print('$e', 'D step %.3f vjp %.3f' % (d['step_ms'], d['unet_vjp_ms']), 'Case4 %.3f it/s' % c['value'])"
done
