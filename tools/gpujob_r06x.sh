# round 6x: after the small-batch CU split and the GroupNorm unroll change: the pipeline tests, the
# GroupNorm-touching parity suites, the driver's bench command and the strong share
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_plan_batch.py tests/test_gpu_knobs.py tests/test_debug_build.py "tests/test_gpu_cfg.py::test_configB_full_256_step_trajectory" > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 5; }
tail -1 $O/tests.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/benchB.json 2> $O/benchB.err || { tail -20 $O/benchB.err; exit 6; }
timeout -k 10 300 python3 bench.py --per-gpu-batch 1 --steps 8 --warmup 2 --no-cpu-baseline > $O/benchB1.json 2> $O/benchB1.err || { tail -20 $O/benchB1.err; exit 7; }
for c in B B1; do python3 -c "import json; d=json.load(open('$O/bench$c.json')); print('$c', d['value'], d['ms_per_step'], d.get('pipeline', {}).get('sample_cus'), d.get('pipeline', {}).get('decode_half_rows', [])[-3:])"; done
