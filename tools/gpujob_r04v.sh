# PMC record of the TrainLoop kernels (Case1 recipe): four counter passes, each its own run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04v; mkdir -p $O
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
         "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAVES" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- python3 tools/kbench.py utrain --batch 16 --size 128 > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 11; }
done
PMC_ALL=1 python3 tools/convpmc.py $O/p1 $O/p2 $O/p3 $O/p4 > $O/r04v_utrain_pmc.txt 2>&1 || true
rm -rf $O/p1 $O/p2 $O/p3 $O/p4
grep -E "wgrad|conv_h|gn_act|absmax|attn_bwd" $O/r04v_utrain_pmc.txt | head -40
