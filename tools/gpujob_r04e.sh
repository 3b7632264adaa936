# in-kernel timestamps of the small-batch U-Net forwards (stamps build) + a parity smoke of the release build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for spec in "b64b1 --size 64 --batch 1" "a32b1 --size 32 --mult 1,2,3,4 --batch 1" "b64b8 --size 64 --batch 8"; do
  set -- $spec; tag=$1; shift
  CFD_LIB=libconfild_hip_stamps.so timeout -k 10 200 python tools/dev/stamps.py "$@" --detail 400 --json $O/$tag.json > $O/$tag.txt 2>&1 || { tail -20 $O/$tag.txt; exit 2; }
  tail -8 $O/$tag.txt
done
