# round 6c: (1) the decoder's in-kernel clock (stamps build) on the whole chip, on its CU half
# alone, and beside the sampler (the pipelined condition); (2) the HEAD PMC record of the
# headline configuration (bench.py config B pipelined, 4 batches): SQ / FETCH / WRITE passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06c; mkdir -p $O
CFD_LIB=libconfild_hip_stamps.so timeout -k 10 300 python3 tools/dev/siren_clock.py --json $O/siren_clock.json > $O/siren_clock.log 2>&1 || { tail -20 $O/siren_clock.log; exit 1; }
cat $O/siren_clock.json
i=0
for P in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  CFD_SAMPLER=1 timeout -s KILL 500 rocprofv3 --pmc $P --output-format csv -d $O/pmc$i -o run -- python3 bench.py --steps 4 --warmup 0 --no-cpu-baseline > $O/pmc$i.log 2>&1 || { tail -5 $O/pmc$i.log; exit $((10+i)); }
  echo "pass $i done"
done
python3 tools/pipe_pmc.py $O/pmc1/run_counter_collection.csv $O/pmc2/run_counter_collection.csv $O/pmc3/run_counter_collection.csv $O/pipe_pmc.json > $O/pipe_pmc.txt 2>&1 || { tail -20 $O/pipe_pmc.txt; ls -R $O | head; exit 20; }
rm -rf $O/pmc1 $O/pmc2 $O/pmc3
cat $O/pipe_pmc.txt
