# DPS timings: config D full loop (B=8), real Case4 384^2 at B=1 and B=8 (50 steps), rocprof stats of Case4 B=1
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py --config D --steps 1 --warmup 1 > gpurun_out/dpsD.json 2> gpurun_out/dpsD.err || { tail -20 gpurun_out/dpsD.err; exit 1; }
cat gpurun_out/dpsD.json
timeout -k 10 300 python3 bench.py --config Case4 --dps-steps 50 --steps 1 --warmup 1 > gpurun_out/case4_b1.json 2> gpurun_out/case4_b1.err || { tail -20 gpurun_out/case4_b1.err; exit 2; }
cat gpurun_out/case4_b1.json
timeout -k 10 400 python3 bench.py --config Case4 --dps-steps 30 --batch 8 --steps 1 --warmup 1 > gpurun_out/case4_b8.json 2> gpurun_out/case4_b8.err || { tail -20 gpurun_out/case4_b8.err; exit 3; }
cat gpurun_out/case4_b8.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_case4 -o run -- python3 bench.py --config Case4 --dps-steps 20 --steps 1 --warmup 1 > gpurun_out/prof_case4.log 2>&1 || { tail -20 gpurun_out/prof_case4.log; exit 4; }
S=$(find gpurun_out/prof_case4 -name "*kernel_stats.csv" | head -1); head -25 $S
