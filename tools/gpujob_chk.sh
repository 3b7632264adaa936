# selected GPU tests then short bench lines (args: pytest targets); BENCH env: bench configs to run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/chk; mkdir -p $O
timeout -k 10 700 python -u -m pytest "$@" -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error|error" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in ${BENCH:-}; do
  case $c in
    E) args="--config E --steps 1 --warmup 0 --no-cpu-baseline";;
    Case4) args="--config Case4 --dps-steps 200 --steps 1 --warmup 1 --no-cpu-baseline";;
    D) args="--config D --steps 2 --warmup 1 --no-cpu-baseline";;
    A) args="--config A --steps 5 --warmup 1 --no-cpu-baseline";;
    B) args="--steps 2 --warmup 1 --no-cpu-baseline";;
    B1) args="--steps 2 --warmup 1 --no-cpu-baseline --per-gpu-batch 1";;
    C) args="--config C --steps 1 --warmup 1 --no-cpu-baseline";;
  esac
  timeout -k 10 400 python3 bench.py $args > $O/bench$c.json 2> $O/bench$c.err || { tail -20 $O/bench$c.err; exit 3; }
  python3 -c "import json; d=json.load(open('$O/bench$c.json')); u=d.get('roofline_unet') or {}; print('$c', round(d['value'],4), d['unit'], round(d['ms_per_step'],2), 'ms/step', 'unet ms/fwd', u.get('ms_per_forward'), 'dec frac', d.get('roofline',{}).get('frac'))"
done
