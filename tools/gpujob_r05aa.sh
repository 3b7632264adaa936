# round 5aa: config E forward, conv plan log + kernel trace in launch order (per-shape durations)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05aa; mkdir -p $O
CFD_CONV_LOG=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof_e -o run -- python3 tools/kbench.py unet --size 128 --batch 8 --bf16 > $O/e.out 2> $O/e.err || { tail -20 $O/e.err; exit 3; }
T=$(find $O/prof_e -name "*kernel_trace.csv" | head -1); gzip -c $T > $O/e_trace.csv.gz; rm -rf $O/prof_e
grep -c CONV $O/e.err
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_cfg.py -k "chain_vs_oracle" > $O/chain.log 2>&1 || { tail -30 $O/chain.log; exit 4; }
grep "chain step\|passed\|failed" $O/chain.log
