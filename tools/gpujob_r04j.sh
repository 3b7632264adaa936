# K1hb two-per-CU register build (CFD_CONV_KHB_OCC) at config E; stamps with per-CU residency
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04j; mkdir -p $O
for r in 1 2; do
for OC in 0 1; do
CFD_CONV_KHB_OCC=$OC timeout -k 10 200 python tools/kbench.py unet --size 128 --batch 8 --unet-compute bf16 > $O/kb.log 2>&1 || { cat $O/kb.log; exit 5; }
echo "KHB_OCC=$OC | $(grep kernel $O/kb.log | cut -c60-200)"
done; done
CFD_LIB=libconfild_hip_stamps.so timeout -k 10 200 python tools/dev/stamps.py --size 128 --batch 8 --bf16 --detail 400 > $O/e128b8.txt 2>&1 || { tail -20 $O/e128b8.txt; exit 3; }
CFD_CONV_KHB_OCC=1 CFD_LIB=libconfild_hip_stamps.so timeout -k 10 200 python tools/dev/stamps.py --size 128 --batch 8 --bf16 --detail 400 > $O/e128b8_occ.txt 2>&1 || { tail -20 $O/e128b8_occ.txt; exit 4; }
CFD_LIB=libconfild_hip_stamps.so timeout -k 10 200 python tools/dev/stamps.py --size 64 --batch 8 --detail 400 > $O/b64b8.txt 2>&1 || { tail -20 $O/b64b8.txt; exit 2; }
tail -5 $O/e128b8.txt; tail -5 $O/e128b8_occ.txt
