# round 5ai: the strong-scaling share on one GPU (1 sample per GPU = config B at 8 GPUs): planned for 1, pipelined
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ai; mkdir -p $O
for a in "--plan-batch 0 --no-pipeline" "--plan-batch 0" "" "--no-pipeline"; do
timeout -k 10 600 python3 bench.py --per-gpu-batch 1 --steps 8 --warmup 1 --no-cpu-baseline $a > $O/s.json 2> $O/s.err || { tail -20 $O/s.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/s.json')); print('per-gpu 1 [$a]', round(d['value'],4), round(d['ms_per_step'],1), d.get('plan_batch'), (d.get('pipeline') or {}).get('sample_ms_per_batch'), (d.get('pipeline') or {}).get('decode_ms_per_batch'))"
done
