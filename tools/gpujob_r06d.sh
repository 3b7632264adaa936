# round 6d: the decoder clock beside the sampler (fixed ordering); HEAD kernel traces of the
# U-Net forwards (config B 64^2 at B = 8 and 1, config E 128^2 bf16 B = 8) and of a config-D DPS
# step; the driver's bench command with the new roofline fields
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 600 python3 tools/libdiff.py libconfild_hip_pre.so libconfild_hip.so > $O/libdiff.json 2> $O/libdiff.err || { cat $O/libdiff.json; tail -20 $O/libdiff.err; exit 9; }
cat $O/libdiff.json
CFD_LIB=libconfild_hip_stamps.so timeout -k 10 300 python3 tools/dev/siren_clock.py --json $O/siren_clock.json > $O/siren_clock.log 2>&1 || { tail -20 $O/siren_clock.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/siren_clock.json')); print({k: (v['clock_ghz_median'], v['launch_ms']) for k, v in d.items() if isinstance(v, dict)}, d['piped'].get('decode_within_sampling'))"
run_trace() {  # name, per, command...
  n=$1; per=$2; shift 2
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_$n -o run -- "$@" > $O/$n.out 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  S=$(find $O/t_$n -name "*kernel_stats.csv" | head -1); cp $S $O/${n}_kernel_stats.csv
  python3 tools/ktrace.py $O/t_$n --per $per --top 30 > $O/${n}_ktrace.txt
  rm -rf $O/t_$n
  head -12 $O/${n}_ktrace.txt
}
run_trace b64b8 12 python3 tools/kbench.py unet --size 64 --batch 8 || exit 2
run_trace b64b1 12 python3 tools/kbench.py unet --size 64 --batch 1 || exit 3
run_trace e128b8 12 python3 tools/kbench.py unet --size 128 --batch 8 --bf16 || exit 4
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 5; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['frac_chip'], d['roofline']['pmc'])"
