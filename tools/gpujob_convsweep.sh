# conv micro-benchmark over split counts for a shape subset (development)
#   bash tools/gpujob_convsweep.sh "<shape substring>" "<splits list>" variant...
set -o pipefail
cd $GRAFT_REPO_ROOT
F=$1; SPL=$2; shift 2
for S in $SPL; do
  echo "== splits $S"
  CX_SHAPES="$F" CX_SPLITS=$S timeout -k 10 120 ./tools/convbench.bin "$@" || exit 1
done
