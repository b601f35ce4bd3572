# Headline-kernel A/B over the rows per load bank (build/abl/lib_pf$v.so, -DLSBM_PF=$v;
# default 4), interleaved, bench.py without the CPU baseline, three passes.
export TMPDIR=/tmp
mkdir -p gpurun_out
for pass in 1 2 3; do
  for v in ${VARIANTS:-4 3 5 6}; do
    if [ $v = 4 ]; then L=""; else L="build/abl/lib_pf$v.so"; fi
    r=$(LSBM_LIB_PATH=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], (d.get('host_staged') or {}).get('mismatches_vs_device_path'))") || exit 1
    echo "pf$v pass $pass: $r" | tee -a gpurun_out/pf_ab.log
  done
done
