#!/bin/bash
# Round profile (run on the GPU box): rocprofv3 kernel trace + stats of the
# bench command, then separate PMC passes for FETCH_SIZE and WRITE_SIZE (never
# combined with sys/runtime traces). Output under gpurun_out/prof_<tag>.
set -euo pipefail
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
for cfg in ${CFGS:-3 2 8 4 6 7 9 10 11}; do
  # 5 warm-up + 30 timed launches; tools/trace_summary.py <csv> 30 averages the same
  # 30 launches bench.py's HIP events time (the stats CSV also counts the warm-up)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c$cfg" -o run -- \
    python3 "$ROOT/bench.py" --config $cfg --steps 30 --warmup 5 --no-cpu-baseline --no-extra --no-e2e \
    > "$OUT/bench_c${cfg}_under_trace.json"
  [ -n "${NO_PMC:-}" ] && continue
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_${ctr}_c$cfg" -o run -- \
      python3 "$ROOT/bench.py" --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-extra --no-e2e \
      > "$OUT/bench_c${cfg}_pmc_$ctr.json"
  done
done
echo done > "$OUT/DONE"
