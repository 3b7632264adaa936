# round 6m: K9t at ring depth 3 with the forward's LDS cut to two workgroups per CU (tape timing,
# expected bit-identical hashes), DPS parity, config D / Case4 lines; where a fresh process's first
# reverse loop spends its extra time (config E and B shapes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 300 python3 tools/dev/tape_bench.py libconfild_hip.so > $O/tape_bench.json 2> $O/tape_bench.err || { tail -20 $O/tape_bench.err; exit 4; }
python3 -c "
import json; d=json.load(open('$O/tape_bench.json'))
for lib, rows in d.items():
    for r in rows: print(lib, {k: (round(v['fwd_ms'],3), round(v['vjp_ms'],3), v['out'], v['gz']) for k, v in r.items()})"
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_dps.py tests/test_gpu_cnftrain.py tests/test_gpu_cfg.py -k "dps or tape or configD or case4 or train" > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 5; }
tail -1 $O/tests.log
timeout -k 10 300 python3 bench.py --config D --steps 2 --warmup 1 --no-cpu-baseline > $O/benchD.json 2> $O/benchD.err || { tail -20 $O/benchD.err; exit 6; }
python3 -c "import json; d=json.load(open('$O/benchD.json')); print('D', d['value'], d['ms_per_step'])"
timeout -k 10 500 python3 bench.py --config Case4 --steps 1 --warmup 1 --no-cpu-baseline > $O/benchCase4.json 2> $O/benchCase4.err || { tail -20 $O/benchCase4.err; exit 7; }
python3 -c "import json; d=json.load(open('$O/benchCase4.json')); print('Case4', d['value'], d['ms_per_step'])"
timeout -k 10 300 python3 tools/dev/first_call.py E > $O/first_E.json 2> $O/first_E.err || { tail -20 $O/first_E.err; exit 8; }
cat $O/first_E.json
timeout -k 10 300 python3 tools/dev/first_call.py B > $O/first_B.json 2> $O/first_B.err || { tail -20 $O/first_B.err; exit 9; }
cat $O/first_B.json
