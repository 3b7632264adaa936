# round 5l: gn2 with 1024-thread workgroups / 256 chunks beyond 128^2: Case4 A/B against the three-kernel path, Case4 parity
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05l; mkdir -p $O
for i in 1 2; do
for v in default 0; do
  if [ $v = default ]; then E=""; else E="CFD_GN2_HW=$v"; fi
  env $E timeout -k 10 200 python3 bench.py --config Case4 --dps-steps 30 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4_$v.json 2> $O/c4_$v.err || { tail -20 $O/c4_$v.err; exit 3; }
  python3 -c "import json; d=json.load(open('$O/c4_$v.json')); print('GN2_HW=$v', round(d['value'],3), round(d['ms_per_step'],3))"
done
done
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cfg.py -k "case4" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 4; }
tail -3 $O/tests.log
