set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "tx_datagram" > gpurun_out/t_dg2.log 2>&1 || { tail -30 gpurun_out/t_dg2.log; exit 1; }
tail -1 gpurun_out/t_dg2.log
YU_TX_FUZZ_ITERS=60 YU_TX_FUZZ_SEED=77 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 500 --timeout-method thread -k "tx_datagram_fuzz" > gpurun_out/t_dg_fuzz60.log 2>&1 || { tail -30 gpurun_out/t_dg_fuzz60.log; exit 1; }
tail -1 gpurun_out/t_dg_fuzz60.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/bench_e2e_tx.json 2> gpurun_out/bench_e2e_tx.err || { tail gpurun_out/bench_e2e_tx.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_e2e_tx.json')); print(d['end_to_end_host_memory'])"
