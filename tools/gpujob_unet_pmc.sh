# rocprofv3 PMC passes over one kbench U-Net run (B = 8, 64x64), summarised by tools/unetpmc.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
         "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAVES" \
         "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d gpurun_out/upmc$i -o run -- python3 tools/kbench.py unet --batch 8 > gpurun_out/upmc$i.log 2>&1 || { tail -5 gpurun_out/upmc$i.log; exit 11; }
done
python3 tools/unetpmc.py gpurun_out/upmc1 gpurun_out/upmc2 gpurun_out/upmc3 gpurun_out/upmc4 gpurun_out/upmc5 > gpurun_out/unet_pmc.txt 2>&1
cat gpurun_out/unet_pmc.txt
