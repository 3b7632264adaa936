# PMC record of the config-B U-Net forward (64^2, B=8, split-f16) at HEAD: four counter
# passes (wave states + MFMA busy; instruction mix; L2 hits; FETCH_SIZE), each its own run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${TAG:-r03k}
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
         "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAVES" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/upmc$i -o run -- python3 tools/kbench.py unet --size 64 --batch 8 > gpurun_out/upmc$i.log 2>&1 || { tail -5 gpurun_out/upmc$i.log; exit 11; }
done
PMC_ALL=1 python3 tools/convpmc.py gpurun_out/upmc1 gpurun_out/upmc2 gpurun_out/upmc3 gpurun_out/upmc4 > gpurun_out/${T}_unet_pmc.txt 2>&1 || true
rm -rf gpurun_out/upmc1 gpurun_out/upmc2 gpurun_out/upmc3 gpurun_out/upmc4
cat gpurun_out/${T}_unet_pmc.txt
