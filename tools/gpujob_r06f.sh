# round 6f: K1s register ring + small-grid tiles for the bf16 (config E) and transposed (DPS input-VJP)
# convolutions too: bit identity against the previous build, then an interleaved A/B of the
# graph-loop step (config E 128^2 B = 8, config B 64^2 B = 8 / 1, config A) and of a config-D DPS step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 600 python3 tools/libdiff.py libconfild_hip_pre.so libconfild_hip_exp.so > $O/libdiff.json 2> $O/libdiff.err || { cat $O/libdiff.json; tail -20 $O/libdiff.err; exit 1; }
cat $O/libdiff.json
i=0
for r in 1 2 3; do
for L in libconfild_hip_pre.so libconfild_hip_exp.so; do
  i=$((i+1))
  CFD_LIB=$L LOOP_MODES=2:4 timeout -k 10 300 python3 tools/loop_probe.py E100 B8 B1 A > $O/k$i.out 2> $O/k$i.err || { tail -20 $O/k$i.err; exit 3; }
  CFD_LIB=$L timeout -k 10 300 python3 tools/kbench.py dps --batch 8 > $O/d$i.out 2> $O/d$i.err || { tail -20 $O/d$i.err; exit 4; }
  python3 -c "
import json
r=[json.loads(l) for l in open('$O/k$i.out') if 'mode' in l]
d=json.loads(open('$O/d$i.out').read().strip().splitlines()[-1])
print('$L', ' '.join('%s=%.3f' % (x['case'], x['ms_per_step']) for x in r), 'dps_step=%.3f vjp=%.3f fwdtape=%.3f siren_fwd=%.3f siren_vjp=%.3f' % (d['step_ms'], d['unet_vjp_ms'], d['unet_fwd_tape_ms'], d['siren_tape_fwd_ms'], d['siren_vjp_ms']))"
done
done
