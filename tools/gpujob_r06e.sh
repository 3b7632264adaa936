# round 6e: in-kernel phase stamps of the U-Net forward at B = 1 and B = 8 (HEAD stamps build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06e; mkdir -p $O
CFD_LIB=libconfild_hip_stamps.so timeout -k 10 200 python3 tools/dev/stamps.py --size 64 --batch 1 > $O/stamps_b64b1.txt 2>&1 || { tail -20 $O/stamps_b64b1.txt; exit 1; }
CFD_LIB=libconfild_hip_stamps.so timeout -k 10 200 python3 tools/dev/stamps.py --size 64 --batch 8 > $O/stamps_b64b8.txt 2>&1 || { tail -20 $O/stamps_b64b8.txt; exit 2; }
tail -6 $O/stamps_b64b1.txt; tail -6 $O/stamps_b64b8.txt
