# Decoder PMC record at HEAD: FETCH_SIZE and WRITE_SIZE passes (separate runs),
# then the MFMA-utilisation pass (decoder + U-Net), each under its own limit.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- python3 tools/kbench.py siren --latents 512 > gpurun_out/pmc_f.log 2>&1 || { tail -5 gpurun_out/pmc_f.log; exit 11; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- python3 tools/kbench.py siren --latents 512 > gpurun_out/pmc_w.log 2>&1 || { tail -5 gpurun_out/pmc_w.log; exit 12; }
F=$(find gpurun_out/pmc_f -name "*counter_collection.csv" | head -1); W=$(find gpurun_out/pmc_w -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py $F $W "siren_split32<" gpurun_out/r02_siren_split32_pmc.json 1628980992 '{"latents": 512, "coords": 262144, "dims": [3, 64, 3, 15, 384]}' || exit 13
cat gpurun_out/r02_siren_split32_pmc.json
bash tools/gpujob_mfma_util.sh
