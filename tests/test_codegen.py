"""Codegen guards (CPU; needs hipcc): properties of the gfx950 machine code
that a kernel's correctness relies on and that the compiler does not promise.

* snappy decoder (lsbm_amd/csrc/snappy_kernels.hip, decode_lanes): the walk
  hands each tag its output offset with an inline `v_writelane_b32` whose lane
  select is in M0 (gfx9's constant bus takes one SGPR besides M0).  M0 is a
  reserved register, so the compiler does not see the inline asm clobber it:
  this checks that no other instruction of the decoder kernels reads or writes
  M0, i.e. that the clobber cannot corrupt a value the compiler keeps there.
"""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _kernel_bodies(asm, name_part):
    """{symbol: [instruction lines]} of the kernels whose symbol contains name_part."""
    out, cur = {}, None
    for line in asm.splitlines():
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur = m.group(1) if name_part in m.group(1) else None
            if cur:
                out[cur] = []
            continue
        if cur is None:
            continue
        if line.strip().startswith("s_endpgm"):
            cur = None
            continue
        ins = line.split(";")[0].strip()
        if ins and not ins.startswith(".") and not ins.endswith(":"):
            out[cur].append(ins)
    return out


@pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which("hipcc")), reason="hipcc not available")
def test_snappy_decoder_m0_only_feeds_writelane(tmp_path):
    src = os.path.join(REPO, "lsbm_amd", "csrc", "snappy_kernels.hip")
    s_file = tmp_path / "snappy_kernels.s"
    subprocess.run([HIPCC if os.path.exists(HIPCC) else "hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    "-w", "--cuda-device-only", "-S", "-o", str(s_file), src], check=True, timeout=600)
    bodies = _kernel_bodies(s_file.read_text(), "snappy_uncompress")
    assert len(bodies) >= 2, "decoder kernels not found in the assembly"
    n_writelane = 0
    for sym, ins in bodies.items():
        for i, line in enumerate(ins):
            if not re.search(r"\bm0\b", line):
                continue
            if line.startswith("s_mov_b32 m0,"):
                assert i + 1 < len(ins) and ins[i + 1].startswith("v_writelane_b32") and \
                    ins[i + 1].endswith("m0"), (sym, line, ins[i + 1:i + 2])
            else:
                assert line.startswith("v_writelane_b32") and line.endswith("m0") and \
                    ins[i - 1].startswith("s_mov_b32 m0,"), (sym, line)
                n_writelane += 1
    assert n_writelane >= 2  # one per decoder kernel at least
