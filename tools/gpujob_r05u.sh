# round 5u: 384^2 / 192^2 128->128 convolutions at one sample: K1s splits 1 / 2, K1x tile variants
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05u; mkdir -p $O
CFD_CONV_KX=0 CX_SHAPES="C4 384^2 conv 128->128" timeout -k 10 300 ./tools/convbench.bin 1 2 20 > $O/a.log 2>&1 || { tail -20 $O/a.log; exit 3; }
cat $O/a.log
CFD_CONV_KX=0 CX_SPLITS=2 CX_SHAPES="C4 384^2 conv 128->128" timeout -k 10 300 ./tools/convbench.bin 30 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 4; }
cat $O/b.log
CFD_CONV_KX=0 CX_SPLITS=2 CX_SHAPES="C4 192^2 conv 128->128" timeout -k 10 300 ./tools/convbench.bin 30 20 > $O/c.log 2>&1 || { tail -20 $O/c.log; exit 5; }
cat $O/c.log
CFD_CONV_KX=0 CFD_CONV_XCD=0 CX_SHAPES="C4 384^2 conv 128->128" timeout -k 10 300 ./tools/convbench.bin > $O/d.log 2>&1 || { tail -20 $O/d.log; exit 6; }
cat $O/d.log
