# round 4, call W: in-place chunk sizes adopted (TXW 48, TX_DATAGRAM fill 40 packets
# per chunk from 64K packets on): the GPU suite, smoke, the bench at the driver's
# settings, a TXW / DG-fill fuzz campaign, and configs 12 / 13 re-profiled
set -o pipefail
mkdir -p gpurun_out
bash tools/verify_round.sh r04w || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r04w_driver.json 2> gpurun_out/bench_r04w_driver.err || { tail gpurun_out/bench_r04w_driver.err; exit 1; }
YU_TX_FUZZ_ITERS=300 YU_TX_FUZZ_SEED=9601 YU_FUZZ_ITERS=3000 YU_FUZZ_SEED=9602 YU_FUZZ_NBIG=70000 \
  timeout -k 10 500 python -u -m pytest -x -q --timeout 480 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "test_tx_datagram_fuzz or test_random_batches_fuzz" > gpurun_out/fuzz_r04w.log 2>&1 || { tail -30 gpurun_out/fuzz_r04w.log; exit 1; }
tail -1 gpurun_out/fuzz_r04w.log
CFGS="12 13" bash tools/profile.sh r04w || exit 1
echo ok
