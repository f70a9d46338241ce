# round 4, call I: closing evidence on the final tree -- the driver's three steps
# (GPU suite, smoke, default bench line), the bench at the driver's settings, and a
# rocprofv3 trace + PMC pass of every bench config
set -o pipefail
mkdir -p gpurun_out
T=r04i
bash tools/verify_round.sh $T || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${T}_driver.json 2> gpurun_out/bench_${T}_driver.err || { tail gpurun_out/bench_${T}_driver.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_${T}_driver.json'));print(d['value'],d['roofline']['frac']);[print(k,v['kernel_avg_us'],v['roofline_frac'],v['kernel']) for k,v in d['other_configs'].items()]"
CFGS="${CFGS:-3 2 8 4}" timeout -k 10 700 bash tools/profile.sh $T || exit 1
echo ok
