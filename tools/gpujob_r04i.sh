# in-kernel stamps at batch 8: config B 64^2 split-f16 and config E 128^2 bf16
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04i; mkdir -p $O
CFD_LIB=libconfild_hip_stamps.so timeout -k 10 200 python tools/dev/stamps.py --size 64 --batch 8 --detail 400 --json $O/b64b8.json > $O/b64b8.txt 2>&1 || { tail -20 $O/b64b8.txt; exit 2; }
tail -6 $O/b64b8.txt
CFD_LIB=libconfild_hip_stamps.so timeout -k 10 200 python tools/dev/stamps.py --size 128 --batch 8 --bf16 --detail 400 --json $O/e128b8.json > $O/e128b8.txt 2>&1 || { tail -20 $O/e128b8.txt; exit 3; }
tail -6 $O/e128b8.txt
