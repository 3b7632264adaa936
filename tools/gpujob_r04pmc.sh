# Decoder PMC record at round-4 HEAD: FETCH_SIZE and WRITE_SIZE passes (separate runs),
# then the MFMA-utilisation pass (decoder + U-Net), each under its own limit; U-Net PMC per kernel family
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04pmc; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- python3 tools/kbench.py siren --latents 512 > $O/pmc_f.log 2>&1 || { tail -5 $O/pmc_f.log; exit 11; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- python3 tools/kbench.py siren --latents 512 > $O/pmc_w.log 2>&1 || { tail -5 $O/pmc_w.log; exit 12; }
F=$(find $O/pmc_f -name "*counter_collection.csv" | head -1); W=$(find $O/pmc_w -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py $F $W "siren_split32<" $O/r04_siren_split32_pmc.json 1628980992 '{"latents": 512, "coords": 262144, "dims": [3, 64, 3, 15, 384]}' || exit 13
cat $O/r04_siren_split32_pmc.json
C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES"
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $O/mu_s -o run -- python3 tools/kbench.py siren --latents 128 > $O/mu_s.log 2>&1 || { tail -5 $O/mu_s.log; exit 14; }
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $O/mu_u -o run -- python3 tools/kbench.py unet --unet-compute split_f16 > $O/mu_u.log 2>&1 || { tail -5 $O/mu_u.log; exit 15; }
python3 tools/mfma_util.py $(find $O/mu_s -name "*counter_collection.csv" | head -1) $(find $O/mu_u -name "*counter_collection.csv" | head -1) --json=$O/r04_mfma_util.json > $O/r04_mfma_util.txt || exit 16
cat $O/r04_mfma_util.txt
