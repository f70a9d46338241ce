# round 4, call N: the whole GPU suite with each ragged measurement override forced
# (parity only: every ragged kernel the selection can be forced onto, the TXW kind
# included), then a longer seeded fuzz campaign on the final tree
set -o pipefail
mkdir -p gpurun_out/forced gpurun_out/fuzz
for f in seg4 seg16 loop rag; do
  YU_RAGGED=$f timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/forced/gpu_tests_r04n_$f.log 2>&1 || { tail -40 gpurun_out/forced/gpu_tests_r04n_$f.log; exit 1; }
  echo "$f: $(tail -1 gpurun_out/forced/gpu_tests_r04n_$f.log)"
done
run() { name=$1; shift; env "$@" timeout -k 10 500 python -u -m pytest -x -v --timeout 480 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "$name" > gpurun_out/fuzz/${name}_r04n.log 2>&1 || { tail -30 gpurun_out/fuzz/${name}_r04n.log; exit 1; }; tail -1 gpurun_out/fuzz/${name}_r04n.log; }
run test_verify_rx_fuzz YU_RX_FUZZ_ITERS=600 YU_RX_FUZZ_SEED=9501 && \
run test_tx_datagram_fuzz YU_TX_FUZZ_ITERS=600 YU_TX_FUZZ_SEED=9502 && \
run test_random_batches_fuzz YU_FUZZ_ITERS=12000 YU_FUZZ_SEED=9503 YU_FUZZ_NBIG=70000 || exit 1
echo ok
