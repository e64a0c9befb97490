set -u
mkdir -p gpurun_out
timeout -k 10 60 ./tools/probe/l2bw.bin 458752 256 512 > gpurun_out/r03g_l2bw.txt 2>&1 &&
timeout -k 10 60 ./tools/probe/l2bw.bin 458752 512 512 >> gpurun_out/r03g_l2bw.txt 2>&1
rc=$?; cat gpurun_out/r03g_l2bw.txt; exit $rc
