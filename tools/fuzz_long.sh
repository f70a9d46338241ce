# Long seeded fuzz campaigns of the GPU parity suite (run on the GPU box). Seeds
# from the environment (defaults: the round-3 campaign), logs under gpurun_out/fuzz/.
set -o pipefail
mkdir -p gpurun_out/fuzz
S=${FUZZ_SEED_BASE:-9300}
run() { name=$1; shift; env "$@" timeout -k 10 280 python -u -m pytest -x -v --timeout 270 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "$name" --durations=3 > gpurun_out/fuzz/${name}_seed$S.log 2>&1 || { tail -30 gpurun_out/fuzz/${name}_seed$S.log; exit 1; }; tail -1 gpurun_out/fuzz/${name}_seed$S.log; }
run test_verify_rx_fuzz YU_RX_FUZZ_ITERS=250 YU_RX_FUZZ_SEED=$((S + 1)) && \
run test_tx_datagram_fuzz YU_TX_FUZZ_ITERS=250 YU_TX_FUZZ_SEED=$((S + 2)) && \
run test_random_batches_fuzz YU_FUZZ_ITERS=3000 YU_FUZZ_SEED=$((S + 3)) YU_FUZZ_NBIG=70000
