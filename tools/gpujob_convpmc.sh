# PMC passes over the conv micro-benchmark (variants given as args)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
         "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAVES" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/cpmc$i -o run -- ./tools/convbench.bin "$@" > gpurun_out/cpmc$i.log 2>&1 || { tail -5 gpurun_out/cpmc$i.log; exit 11; }
done
python3 tools/convpmc.py gpurun_out/cpmc1 gpurun_out/cpmc2 gpurun_out/cpmc3 gpurun_out/cpmc4 > gpurun_out/cpmc_summary.txt 2>&1 || true
cat gpurun_out/cpmc_summary.txt | head -80
