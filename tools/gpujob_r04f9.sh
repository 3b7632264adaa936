# round-end in-kernel stamps (B=1 and B=8 64^2, config E) on the final sources
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04f9; mkdir -p $O
for spec in "b64b1 --size 64 --batch 1" "b64b8 --size 64 --batch 8" "e128b8 --size 128 --batch 8 --bf16"; do
  set -- $spec; tag=$1; shift
  CFD_LIB=libconfild_hip_stamps.so timeout -k 10 200 python tools/dev/stamps.py "$@" --detail 400 > $O/$tag.txt 2>&1 || { tail -20 $O/$tag.txt; exit 2; }
  tail -5 $O/$tag.txt
done
