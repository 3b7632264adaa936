# conv micro-benchmark: K1s (shipped) vs K1x variants on the config-B shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 ./tools/convbench.bin "$@" > gpurun_out/convbench.log 2>&1; RC=$?
cat gpurun_out/convbench.log
exit $RC
