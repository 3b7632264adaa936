# round 5al: HEAD U-Net PMC record (config B forward, 64^2 B = 8, split-f16): four counter passes + kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05al; mkdir -p $O
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
         "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAVES" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/upmc$i -o run -- python3 tools/kbench.py unet --size 64 --batch 8 > $O/upmc$i.log 2>&1 || { tail -5 $O/upmc$i.log; exit 11; }
done
python3 tools/unetpmc.py $O/upmc1 $O/upmc2 $O/upmc3 $O/upmc4 > $O/unet_b64b8_pmc.txt 2>&1 || true
rm -rf $O/upmc1 $O/upmc2 $O/upmc3 $O/upmc4
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/kbench.py unet --size 64 --batch 8 > $O/kb.out 2> $O/kb.err || { tail -5 $O/kb.err; exit 12; }
S=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $S $O/unet_b64b8_kernel_stats.csv; rm -rf $O/prof
head -40 $O/unet_b64b8_pmc.txt
