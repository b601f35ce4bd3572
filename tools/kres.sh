#!/bin/bash
# Register / spill / scratch summary of a HIP source's kernels (gfx950).
#   tools/kres.sh lsbm_amd/csrc/crc32c_stream.hip [extra hipcc flags]
f=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o /dev/null "$f" "$@" \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
cur = None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m: cur = m.group(1); print(cur[:70], end=""); continue
    for k in ("VGPRs:", "VGPRs Spill:", "ScratchSize \\[bytes/lane\\]:", "Occupancy \\[waves/SIMD\\]:"):
        m = re.search(k + r" (\d+)", line)
        if m: print(" ", k.replace("\\", "").split()[0], m.group(1), end="")
    if "LDS Size" in line: print()
'
