# round 6r: key chunks bounded to small grids; config A timed and pinned at planned batch 1:
# parity suites, the config-A line, the 8-GPU strong share on one GPU
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06r; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_plan_batch.py tests/test_gpu_dps.py "tests/test_gpu_cfg.py::test_configA_ddim50_and_decode_end_to_end" "tests/test_gpu_cfg.py::test_configB_full_256_step_trajectory" tests/test_gpu_knobs.py tests/test_gpu_pipeline.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 5; }
tail -1 $O/tests.log
timeout -k 10 300 python3 bench.py --config A --steps 5 --warmup 1 > $O/benchA.json 2> $O/benchA.err || { tail -20 $O/benchA.err; exit 6; }
python3 -c "import json; d=json.load(open('$O/benchA.json')); print('A', d['value'], d['ms_per_step'], d['roofline_unet']['ms_per_forward'], d['config'].get('plan_batch'), d['cpu_baseline'] and d['cpu_baseline']['value'])"
timeout -k 10 300 python3 bench.py --per-gpu-batch 1 --steps 8 --warmup 2 --no-cpu-baseline > $O/benchB1.json 2> $O/benchB1.err || { tail -20 $O/benchB1.err; exit 7; }
python3 -c "import json; d=json.load(open('$O/benchB1.json')); print('B1', d['value'], d['ms_per_step'])"
