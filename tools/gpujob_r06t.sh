# round 6t: kernel trace of config B's U-Net on one CU half (128 CUs), 2 x 16 graph-loop steps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06t; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_h -o run -- python3 tools/dev/half_chip_unet.py 128 > $O/h.out 2> $O/h.err || { tail -5 $O/h.err; exit 2; }
python3 tools/ktrace.py $O/t_h --per 32 --top 60 > $O/half128_ktrace.txt; rm -rf $O/t_h
cat $O/half128_ktrace.txt
