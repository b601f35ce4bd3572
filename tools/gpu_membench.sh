set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 ./build/membench 4 > gpurun_out/membench4.txt 2>&1 && \
timeout -k 10 300 ./build/membench 32 > gpurun_out/membench32.txt 2>&1
rc=$?
cat gpurun_out/membench4.txt gpurun_out/membench32.txt
exit $rc
