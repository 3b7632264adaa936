# round 5p: Case4 (B = 1) convolution shapes: K1s (planner splits, nominal batch 8 / 2) vs K1h / K1x (auto splits)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05p; mkdir -p $O
CFD_CONV_KX=0 CX_SHAPES="C4" timeout -k 10 300 ./tools/convbench.bin 20 2 > $O/cb8.log 2>&1 || { tail -20 $O/cb8.log; exit 3; }
cat $O/cb8.log
CFD_PLAN_B=2 CFD_CONV_KX=0 CX_SHAPES="C4" timeout -k 10 300 ./tools/convbench.bin 20 > $O/cb2.log 2>&1 || { tail -20 $O/cb2.log; exit 4; }
cat $O/cb2.log
