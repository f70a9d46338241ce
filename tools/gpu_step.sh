# round 4, call O: round-end verification on the final tree (GPU suite, smoke,
# default bench line), the driver's bench settings, and a profile of config 12
# (its fill kernel loads plainly since r04i)
set -o pipefail
bash tools/verify_round.sh r04o || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r04o_driver.json 2> gpurun_out/bench_r04o_driver.err || { tail gpurun_out/bench_r04o_driver.err; exit 1; }
CFGS="12" bash tools/profile.sh r04o || exit 1
echo ok
