set -o pipefail
mkdir -p gpurun_out
run() {  # tag, env..., config
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra --no-e2e > gpurun_out/eager_$tag.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/eager_$tag.json'));print('$tag', d['roofline']['kernel_avg_us'], d['ms_per_step'])"
}
bench_cfg() { local tag=$1 c=$2; shift 2; env "$@" timeout -k 10 200 python bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-extra --no-e2e > gpurun_out/eager_$tag.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/eager_$tag.json'));print('$tag', d['roofline']['kernel_avg_us'], d['ms_per_step'])"; }
bench_cfg c11 11
bench_cfg c11_b16 11 YU_BLOCKS_PER_CU=16
bench_cfg c11_b4 11 YU_BLOCKS_PER_CU=4
bench_cfg c6 6
bench_cfg c6_b16 6 YU_BLOCKS_PER_CU=16
timeout -k 10 100 tools/kbench 15 | tail -1
YU_BLOCKS_PER_CU=16 timeout -k 10 100 tools/kbench 15 | tail -1
