# Round-1 bench + profiles: bench.py line, rocprofv3 kernel stats of the same
# command, FETCH/WRITE PMC passes of the dominant decoder kernel.
set -o pipefail
TAG=${TAG:-r01d}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/profiles_new
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 14; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || { tail -20 gpurun_out/prof_bench.log; exit 15; }
S=$(find gpurun_out/prof_bench -name "*kernel_stats.csv" | head -1); cp $S gpurun_out/profiles_new/${TAG}_bench_kernel_stats.csv; head -12 $S
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- python3 tools/kbench.py siren --latents 512 > gpurun_out/pmc_f.log 2>&1 || { tail -5 gpurun_out/pmc_f.log; exit 11; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- python3 tools/kbench.py siren --latents 512 > gpurun_out/pmc_w.log 2>&1 || { tail -5 gpurun_out/pmc_w.log; exit 12; }
F=$(find gpurun_out/pmc_f -name "*counter_collection.csv" | head -1); W=$(find gpurun_out/pmc_w -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py $F $W "siren_split32<" gpurun_out/profiles_new/r01_siren_split32_pmc.json 1628980992 '{"latents": 512, "coords": 262144, "dims": [3, 64, 3, 15, 384]}' || exit 13
echo done
