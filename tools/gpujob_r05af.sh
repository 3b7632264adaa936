# round 5af: config B pipelined (decode of batch k-1 beside the sampling of batch k) vs sequential, same box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05af; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_streams.py > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 2; }
tail -1 $O/t.log
timeout -k 10 900 python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline > $O/pipe.json 2> $O/pipe.err || { tail -20 $O/pipe.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/pipe.json')); print('pipelined', round(d['value'],4), round(d['ms_per_step'],1), d.get('pipeline'), d['roofline']['frac'], d['roofline_unet']['frac'])"
timeout -k 10 900 python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-pipeline > $O/seq.json 2> $O/seq.err || { tail -20 $O/seq.err; exit 4; }
python3 -c "import json; d=json.load(open('$O/seq.json')); print('sequential', round(d['value'],4), round(d['ms_per_step'],1), d['roofline']['frac'])"
