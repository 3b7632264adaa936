# round 5n: which switch makes config D batched == single chains under K9s
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05n; mkdir -p $O
for e in "CFD_ATTN_BWD_SPLIT=0" "CFD_ATTN_BWD_W8=0" "CFD_ATTN_XCD=0" "CFD_ATTN_BWD_W8=0 CFD_ATTN_XCD=0"; do
  env $e timeout -k 10 300 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_cfg.py -k "configD_batched" > $O/t.log 2>&1
  rc=$?
  echo "$e rc=$rc $(tail -1 $O/t.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
done
