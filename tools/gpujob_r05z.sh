# round 5z: config E bench line with warmup (the checkpoint's E ran cold)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05z; mkdir -p $O
timeout -k 10 600 python3 bench.py --config E --steps 2 --warmup 1 > $O/benchE.json 2> $O/benchE.err || { tail -20 $O/benchE.err; exit 7; }
python3 -c "import json; d=json.load(open('$O/benchE.json')); print('E', round(d['value'],3), round(d['ms_per_step'],1), d['roofline_unet']['ms_per_forward'], d['roofline']['frac'])"
