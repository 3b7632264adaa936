# GroupNorm micro-benchmark at B = 8 and 16, shipped and variant paths (development)
set -o pipefail
cd $GRAFT_REPO_ROOT
for E in "CFD_NONE=1" "CFD_GN_NT1024=0" "CFD_GN_FUSED=0"; do
  echo "== $E"
  env $E timeout -k 10 60 ./tools/gnbench.bin 8 || exit 1
  env $E timeout -k 10 60 ./tools/gnbench.bin 16 || exit 1
done
