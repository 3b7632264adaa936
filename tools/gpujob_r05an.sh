# round 5an: split-K slab of the VJP's GroupNorm-feeding convolutions reduced inside the GroupNorm
# backward statistics pass (CFD_VJP_GNFUSE): parity, config D / Case4 A/B, then the pipeline CU split at 20 steps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05an; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dps.py tests/test_gpu_plan_batch.py tests/test_gpu_unet_train.py > $O/tests1.log 2>&1 || { tail -40 $O/tests1.log; exit 3; }
tail -2 $O/tests1.log
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cfg.py -k "configD or case4 or Case4" > $O/tests2.log 2>&1 || { tail -40 $O/tests2.log; exit 4; }
tail -2 $O/tests2.log
for v in 1 0 1 0; do
  CFD_VJP_GNFUSE=$v timeout -k 10 200 python3 tools/kbench.py dps --batch 8 > $O/d_$v.out 2> $O/d_$v.err || { tail -20 $O/d_$v.err; exit 5; }
  echo "gnfuse=$v $(cat $O/d_$v.out)"
done
for v in 1 0 1 0; do
  CFD_VJP_GNFUSE=$v timeout -k 10 200 python3 bench.py --config Case4 --dps-steps 30 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4ab.json 2> $O/c4ab.err || { tail -20 $O/c4ab.err; exit 8; }
  python3 -c "import json; d=json.load(open('$O/c4ab.json')); print('Case4 gnfuse=$v', round(d['value'],3), round(d['ms_per_step'],3))"
done
timeout -k 10 300 python3 bench.py --config D --steps 2 --warmup 1 > $O/benchD.json 2> $O/benchD.err || { tail -20 $O/benchD.err; exit 9; }
python3 -c "import json; d=json.load(open('$O/benchD.json')); print('D', round(d['value'],3), d['unit'], round(d['ms_per_step'],2))"
for h in 96 128; do
CFD_PIPE_SAMPLE_CUS=$h timeout -k 10 600 python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/p$h.json 2> $O/p$h.err || { tail -20 $O/p$h.err; exit 10; }
python3 -c "import json; d=json.load(open('$O/p$h.json')); p=d['pipeline']; print('sample CUs $h', round(d['value'],4), round(d['ms_per_step'],1), round(p['sample_ms_per_batch']), round(p['decode_ms_per_batch']))"
done
