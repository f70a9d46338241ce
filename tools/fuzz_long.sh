set -o pipefail
mkdir -p gpurun_out/fuzz
run() { name=$1; shift; env "$@" timeout -k 10 280 python -u -m pytest -x -v --timeout 270 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "$name" --durations=3 > gpurun_out/fuzz/$name.log 2>&1 || { tail -30 gpurun_out/fuzz/$name.log; exit 1; }; tail -1 gpurun_out/fuzz/$name.log; }
run test_verify_rx_fuzz YU_RX_FUZZ_ITERS=250 YU_RX_FUZZ_SEED=9001 && \
run test_tx_datagram_fuzz YU_TX_FUZZ_ITERS=250 YU_TX_FUZZ_SEED=9002 && \
run test_random_batches_fuzz YU_FUZZ_ITERS=4000 YU_FUZZ_SEED=9003
