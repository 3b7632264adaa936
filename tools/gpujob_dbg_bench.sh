# Bounds-checked build test, then one default config-B bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r02l}
timeout -k 10 300 python -u -m pytest tests/test_debug_build.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/dbg.log 2>&1 || { tail -20 gpurun_out/dbg.log; exit 1; }
tail -n 1 gpurun_out/dbg.log
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 2; }
python3 - <<PY
import json
d = json.load(open("gpurun_out/bench_$TAG.json")); r = d["roofline"]; u = d["roofline_unet"]
print(d["value"], r["launch_ms"], r["frac"], r["frac_sustained"], u["ms_per_forward"])
PY
