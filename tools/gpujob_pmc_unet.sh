set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmc_u1 -o run -- python3 tools/kbench.py unet --unet-compute split_f16 > gpurun_out/pmc_u1.log 2>&1 || { tail -5 gpurun_out/pmc_u1.log; exit 11; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAVES --output-format csv -d gpurun_out/pmc_u2 -o run -- python3 tools/kbench.py unet --unet-compute split_f16 > gpurun_out/pmc_u2.log 2>&1 || { tail -5 gpurun_out/pmc_u2.log; exit 12; }
echo done
