# conv micro-benchmark, K1s under two environments (A/B of an env switch):
#   bash tools/gpujob_convbench_env.sh "ENV_A=.." "ENV_B=.."
set -o pipefail
cd $GRAFT_REPO_ROOT
env $1 timeout -k 10 300 ./tools/convbench.bin ${3:-20} > gpurun_out/convbench_a.log 2>&1 || exit 1
env $2 timeout -k 10 300 ./tools/convbench.bin ${3:-20} > gpurun_out/convbench_b.log 2>&1 || exit 2
env $1 timeout -k 10 300 ./tools/convbench.bin ${3:-20} > gpurun_out/convbench_a2.log 2>&1 || exit 3
paste -d'|' <(grep K1s gpurun_out/convbench_a.log | cut -c1-110) <(grep K1s gpurun_out/convbench_b.log | cut -c80-110) <(grep K1s gpurun_out/convbench_a2.log | cut -c80-110)
