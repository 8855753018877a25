bash tools/gpu/sweep.sh "crc32 qsort" "64 16 8 4 1" "4 8"
