# read probe: k_seg's 8 KiB tile stream, u-major (k_seg's layout) vs lane-major loads
set -o pipefail
mkdir -p gpurun_out
PROBE_TILES=1 timeout -k 10 120 tools/hbm_probe 126000000 17 > gpurun_out/hbm_probe_tiles_126MB.log 2>&1 || { tail gpurun_out/hbm_probe_tiles_126MB.log; exit 1; }
PROBE_TILES=1 timeout -k 10 120 tools/hbm_probe 1583349760 2 > gpurun_out/hbm_probe_tiles_1.58GB.log 2>&1 || { tail gpurun_out/hbm_probe_tiles_1.58GB.log; exit 1; }
grep "round 1" gpurun_out/hbm_probe_tiles_126MB.log gpurun_out/hbm_probe_tiles_1.58GB.log
