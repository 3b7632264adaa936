# same-box A/B of an environment switch on the U-Net forward (kbench) and the full bench line
#   bash tools/gpujob_ab_bench.sh "ENV_A=.." "ENV_B=.."
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
for E in "$1" "$2"; do
  env $E timeout -k 10 200 python3 tools/kbench.py unet --batch 8 > gpurun_out/ab_unet.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
  echo "$E $(cat gpurun_out/ab_unet.json)"
done
done
for E in "$1" "$2"; do
  env $E timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/ab_bench.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 2; }
  echo "$E $(python3 -c "import json;d=json.load(open('gpurun_out/ab_bench.json'));print(round(d['value'],4),'fields/s unet_ms/fwd',round(d['roofline_unet']['ms_per_forward'],3),'dec_ms',round(d['roofline']['launch_ms'],1))")"
done
