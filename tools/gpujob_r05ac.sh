set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05ac
timeout -k 10 200 python3 tools/dev/sync_probe.py > gpurun_out/r05ac/sync.log 2>&1 || { tail -30 gpurun_out/r05ac/sync.log; exit 3; }
grep -c "SYNC:" gpurun_out/r05ac/sync.log
