# Host -> host rates of the C++ layers (build/bench_host_layers, built in the build container).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 build/bench_host_layers ${TABLES:-1000} ${WAL_MB:-1024} > gpurun_out/host_layers.log 2>&1
rc=$?; echo "host_layers rc=$rc"; cat gpurun_out/host_layers.log | cut -c1-300
exit $rc
