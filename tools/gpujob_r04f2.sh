# round-4 final checkpoint, part 2 (round end): every configuration's bench line with its cpu_baseline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04f2; mkdir -p $O
for cfg in B A C D E; do
  timeout -k 10 600 python bench.py --config $cfg > $O/bench$cfg.json 2> $O/bench$cfg.err || { echo BENCHFAIL $cfg; tail -20 $O/bench$cfg.err; exit 3; }
  cat $O/bench$cfg.json
done
timeout -k 10 600 python bench.py --config Case4 --dps-steps 1000 > $O/benchCase4.json 2> $O/benchCase4.err || { echo BENCHFAIL Case4; tail -20 $O/benchCase4.err; exit 3; }
cat $O/benchCase4.json
timeout -k 10 300 python3 tools/kbench.py utrain --batch 16 --size 128 > $O/utrain.json 2> $O/utrain.err || { tail -20 $O/utrain.err; exit 4; }
cat $O/utrain.json
