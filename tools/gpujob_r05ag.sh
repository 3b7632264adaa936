# round 5ag: config B pipeline CU split (sampling CUs 96 / 112 / 128 / 144), 8 steps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ag; mkdir -p $O
for h in 96 112 128 144; do
CFD_PIPE_SAMPLE_CUS=$h timeout -k 10 900 python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline > $O/p$h.json 2> $O/p$h.err || { tail -20 $O/p$h.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/p$h.json')); p=d['pipeline']; print('sample CUs $h', round(d['value'],4), round(d['ms_per_step'],1), round(p['sample_ms_per_batch']), round(p['decode_ms_per_batch']))"
done
