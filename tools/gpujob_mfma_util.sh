# MFMA utilisation and effective clock of the decoder (K7t) and the U-Net kernels:
# one rocprofv3 PMC pass each (GRBM_GUI_ACTIVE + SQ_VALU_MFMA_BUSY_CYCLES + SQ_INSTS_MFMA)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES"
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d gpurun_out/mu_s -o run -- python3 tools/kbench.py siren --latents 128 > gpurun_out/mu_s.log 2>&1 || { tail -5 gpurun_out/mu_s.log; exit 11; }
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d gpurun_out/mu_u -o run -- python3 tools/kbench.py unet --unet-compute split_f16 > gpurun_out/mu_u.log 2>&1 || { tail -5 gpurun_out/mu_u.log; exit 12; }
python3 tools/mfma_util.py gpurun_out/mu_s/run_counter_collection.csv gpurun_out/mu_u/run_counter_collection.csv --json=gpurun_out/mfma_util.json > gpurun_out/mfma_util.txt || exit 13
cat gpurun_out/mfma_util.txt
