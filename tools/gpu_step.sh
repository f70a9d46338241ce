# round 4, call G: long seeded fuzz campaigns on the final kernels (incl. the in-place
# TXW kind at 64-packet chunks, YU_FUZZ_NBIG=70000), and the driver's own launch form
# (torch.distributed.run, 8 ranks) rehearsed on the one card
set -o pipefail
mkdir -p gpurun_out
FUZZ_SEED_BASE=9400 bash tools/fuzz_long.sh || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 8 --steps 20 --warmup 5 > gpurun_out/bench_r04g_torchrun_8ranks.json 2> gpurun_out/bench_r04g_torchrun_8ranks.err || { tail -20 gpurun_out/bench_r04g_torchrun_8ranks.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_r04g_torchrun_8ranks.json'));print(d['n_gpus'],d['value'],d['config']['parallelism'],[p['GiB_s'] for p in d['per_gpu']])"
echo ok
