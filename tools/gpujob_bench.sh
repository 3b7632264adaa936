set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- python3 tools/kbench.py siren --latents 512 > gpurun_out/pmc_f.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- python3 tools/kbench.py siren --latents 512 > gpurun_out/pmc_w.log 2>&1 || exit 12
F=$(find gpurun_out/pmc_f -name "*counter_collection.csv" | head -1); W=$(find gpurun_out/pmc_w -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py $F $W siren_fused profiles/r01_siren_pmc.json 1628980992 '{"latents": 512, "coords": 262144, "dims": [3, 64, 3, 15, 384]}' || exit 13
cp $F profiles/r01_siren_pmc_fetch.csv; cp $W profiles/r01_siren_pmc_write.csv
mkdir -p gpurun_out/profiles_new && cp profiles/r01_siren_pmc* gpurun_out/profiles_new/
timeout -k 10 900 python3 bench.py > gpurun_out/bench_r01c.json 2> gpurun_out/bench_r01c.err || exit 14
cat gpurun_out/bench_r01c.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit 15
echo done
