# same-box A/B of an environment switch on the DPS benches (config D, Case4 B=1 and B=8)
#   bash tools/gpujob_dps_ab.sh "ENV_A=.." "ENV_B=.."
set -o pipefail
cd $GRAFT_REPO_ROOT
for E in "$1" "$2"; do
  env $E timeout -k 10 300 python3 bench.py --config D --steps 1 --warmup 1 > gpurun_out/ab_d.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
  env $E timeout -k 10 300 python3 bench.py --config Case4 --dps-steps 50 --steps 1 --warmup 1 > gpurun_out/ab_c1.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 2; }
  env $E timeout -k 10 400 python3 bench.py --config Case4 --dps-steps 30 --batch 8 --steps 1 --warmup 1 > gpurun_out/ab_c8.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 3; }
  echo "$E D $(python3 -c "import json;print(round(json.load(open('gpurun_out/ab_d.json'))['value'],1))") it/s, Case4 B=1 $(python3 -c "import json;print(round(json.load(open('gpurun_out/ab_c1.json'))['value'],2))"), B=8 $(python3 -c "import json;print(round(json.load(open('gpurun_out/ab_c8.json'))['value'],2))")"
done
