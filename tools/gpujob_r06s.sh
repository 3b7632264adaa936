# round 6s: K1hb (config E's bf16 3x3 convolutions) on 128-pixel blocks of 4 waves, two workgroups
# per CU (development build bm128): bit identity against the shipped build, interleaved A/B of
# config E's graph-loop step, kernel trace of the 128^2 forward
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s; mkdir -p $O
timeout -k 10 600 python3 tools/libdiff.py libconfild_hip.so libconfild_hip_bm128.so > $O/libdiff.json 2> $O/libdiff.err || { cat $O/libdiff.json; tail -20 $O/libdiff.err; exit 1; }
cat $O/libdiff.json
i=0
for r in 1 2 3; do
for L in libconfild_hip.so libconfild_hip_bm128.so; do
  i=$((i+1))
  CFD_LIB=$L LOOP_MODES=2:4 timeout -k 10 300 python3 tools/loop_probe.py E100 > $O/k$i.out 2> $O/k$i.err || { tail -20 $O/k$i.err; exit 3; }
  python3 -c "
import json
r=[json.loads(l) for l in open('$O/k$i.out') if 'mode' in l]
print('$L', ' '.join('%s=%.3f' % (x['case'], x['ms_per_step']) for x in r))"
done
done
CFD_LIB=libconfild_hip_bm128.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_e -o run -- python3 tools/kbench.py unet --size 128 --batch 8 --bf16 > $O/e.out 2> $O/e.err || { tail -5 $O/e.err; exit 5; }
python3 tools/ktrace.py $O/t_e --per 12 --top 30 > $O/e128b8_bm128_ktrace.txt; rm -rf $O/t_e
head -26 $O/e128b8_bm128_ktrace.txt
