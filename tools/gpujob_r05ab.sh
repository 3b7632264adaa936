set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ab; mkdir -p $O
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/dev/siren_upload_probe.py > $O/p.out 2> $O/p.err || { tail -20 $O/p.err; exit 3; }
cat $O/p.out
for f in $(find $O/prof -name "*.csv"); do gzip -c $f > $O/$(basename $f).gz; done; rm -rf $O/prof
ls $O
