# round 5ad: cached normaliser device params (no stream syncs in the SIREN tape): config D step, Case4, DPS tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ad; mkdir -p $O
timeout -k 10 200 python3 tools/dev/sync_probe.py > $O/sync.log 2>&1 || { tail -30 $O/sync.log; exit 3; }
echo "syncs: $(grep -c 'SYNC: called' $O/sync.log)"
for i in 1 2; do
timeout -k 10 200 python3 tools/kbench.py dps --batch 8 > $O/d.out 2> $O/d.err || { tail -20 $O/d.err; exit 5; }
python3 -c "import json; d=json.load(open('$O/d.out')); print('D step', round(d['step_ms'],3), 'vjp', round(d['unet_vjp_ms'],3))"
done
timeout -k 10 300 python3 bench.py --config D --steps 2 --warmup 1 --no-cpu-baseline > $O/benchD.json 2> $O/benchD.err || { tail -20 $O/benchD.err; exit 6; }
python3 -c "import json; d=json.load(open('$O/benchD.json')); print('D', round(d['value'],2), round(d['ms_per_step'],3))"
timeout -k 10 200 python3 bench.py --config Case4 --dps-steps 30 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 7; }
python3 -c "import json; d=json.load(open('$O/c4.json')); print('Case4', round(d['value'],3), round(d['ms_per_step'],3))"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dps.py tests/test_gpu_cfg.py -k "dps or vjp or configD or case4 or siren" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 8; }
tail -1 $O/tests.log
