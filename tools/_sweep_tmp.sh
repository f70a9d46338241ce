set -o pipefail
timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --steps 20 > gpurun_out/bench_rx.json 2>gpurun_out/bench_rx.err || { tail gpurun_out/bench_rx.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_rx.json').read().strip().splitlines()[-1]);print({k:v for k,v in d['end_to_end_host_memory'].items() if 'burst' in k})"
YU_RAGGED=seg8 timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --steps 20 > gpurun_out/bench_rx_seg.json 2>/dev/null
python3 -c "import json;d=json.loads(open('gpurun_out/bench_rx_seg.json').read().strip().splitlines()[-1]);print('seg8', {k:v for k,v in d['end_to_end_host_memory'].items() if 'rx_burst' in k})"
