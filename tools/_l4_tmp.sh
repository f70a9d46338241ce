tools/ab.sh "2" "2 YU_VARIANT=k_lane<4>" "14 KB_LEN=64" "14 KB_LEN=64 YU_VARIANT=k_lane<4>" "14 KB_LEN=48 YU_VARIANT=k_lane<4>" "14 KB_LEN=48" "14 KB_LEN=64 KB_FILL=1" "14 KB_LEN=64 KB_FILL=1 YU_VARIANT=k_lane<4>" "2" "2 YU_VARIANT=k_lane<4>" > gpurun_out/l4_ab.log 2>&1
grep -v "round 0" gpurun_out/l4_ab.log
