# Host-layer staging A/B: build/abl/<v>/liblsbm_crc32c.so built with other
# LSBM_HOST_STAGES / LSBM_HOST_CHUNK_MB (host_session.h), picked up through
# LD_LIBRARY_PATH by build/bench_host_layers; two interleaved passes.
export TMPDIR=/tmp
mkdir -p gpurun_out
for pass in 1 2; do
  for v in base ${VARIANTS:-st4 c32 c128}; do
    echo "== $v pass $pass" >> gpurun_out/host_stages_ab.log
    if [ $v = base ]; then P=""; else P="build/abl/$v"; fi
    LD_LIBRARY_PATH=$P${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 300 build/bench_host_layers ${TABLES:-1000} 1024 >> gpurun_out/host_stages_ab.log 2>&1 || exit 1
  done
done
