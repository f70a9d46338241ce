set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke3.log 2>&1 || { tail gpurun_out/smoke3.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench_final3.json 2> gpurun_out/bench_final3.err || { tail gpurun_out/bench_final3.err; exit 1; }
CFGS="2 8 10" timeout -k 10 600 bash tools/profile.sh final3 > gpurun_out/profile_final3.log 2>&1 || { tail gpurun_out/profile_final3.log; exit 1; }
echo all ok
