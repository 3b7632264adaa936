# round 5m: split-f16 attention backward (K9s): DPS / training parity, config D step A/B, kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dps.py tests/test_gpu_unet_train.py > $O/tests1.log 2>&1 || { tail -40 $O/tests1.log; exit 3; }
tail -2 $O/tests1.log
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cfg.py -k "configD or case4" > $O/tests2.log 2>&1 || { tail -40 $O/tests2.log; exit 4; }
tail -2 $O/tests2.log
for v in 1 0 1; do
  CFD_ATTN_BWD_SPLIT=$v timeout -k 10 200 python3 tools/kbench.py dps --batch 8 > $O/d_$v.out 2> $O/d_$v.err || { tail -20 $O/d_$v.err; exit 5; }
  echo "split=$v $(cat $O/d_$v.out)"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_d -o run -- python3 tools/kbench.py dps --batch 8 > $O/dprof.out 2> $O/dprof.err || { tail -20 $O/dprof.err; exit 6; }
S=$(find $O/prof_d -name "*kernel_stats.csv" | head -1); cp $S $O/d_stats.csv
T=$(find $O/prof_d -name "*kernel_trace.csv" | head -1); gzip -c $T > $O/d_trace.csv.gz; rm -rf $O/prof_d
CFD_CONV_LOG=1 timeout -k 10 200 python3 bench.py --config Case4 --dps-steps 1 --steps 1 --warmup 0 --no-cpu-baseline > $O/c4log.out 2> $O/c4log.err || { tail -20 $O/c4log.err; exit 7; }
for e in "X=0" "CFD_GNB2=0" "CFD_CONV_KH=0" "CFD_CONV_KX=0" "X=0"; do
  env $e timeout -k 10 200 python3 bench.py --config Case4 --dps-steps 30 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4ab.json 2> $O/c4ab.err || { tail -20 $O/c4ab.err; exit 8; }
  python3 -c "import json; d=json.load(open('$O/c4ab.json')); print('$e', round(d['value'],3), round(d['ms_per_step'],3))"
done
timeout -k 10 300 python3 bench.py --config D --steps 2 --warmup 1 > $O/benchD.json 2> $O/benchD.err || { tail -20 $O/benchD.err; exit 9; }
python3 -c "import json; d=json.load(open('$O/benchD.json')); print('D', round(d['value'],3), d['unit'], round(d['ms_per_step'],2))"
