"""Codegen guards (CPU; needs hipcc): properties of the gfx950 machine code
that a kernel's correctness relies on and that the compiler does not promise.

* snappy decoder (lsbm_amd/csrc/snappy_kernels.hip, decode_lanes): the walk
  hands each tag its output offset with an inline `v_writelane_b32` whose lane
  select is in M0 (gfx9's constant bus takes one SGPR besides M0).  M0 is a
  reserved register, so the compiler does not see the inline asm clobber it:
  this checks that no instruction of the decoder kernels outside the inline
  asm blocks (the walk: `s_and_b32 m0` / `v_writelane_b32 .., m0` /
  `v_readlane_b32 .., m0`) reads or writes M0, i.e. that the clobber cannot
  corrupt a value the compiler keeps there.
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
        if ";;#ASMSTART" in line or ";;#ASMEND" in line:
            out[cur].append(line.strip())
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
    for sym, ins in bodies.items():
        in_asm, n_lane_m0 = False, 0
        for line in ins:
            if line.startswith(";;#ASMSTART"):
                in_asm = True
            elif line.startswith(";;#ASMEND"):
                in_asm = False
            elif re.search(r"\bm0\b", line):
                assert in_asm, (sym, "M0 used outside the inline asm", line)
                n_lane_m0 += line.startswith(("v_writelane_b32", "v_readlane_b32"))
        assert n_lane_m0 >= 1, (sym, "no lane select through M0 found")


@pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which("hipcc")), reason="hipcc not available")
def test_crc_kernels_do_not_spill(tmp_path):
    """The fixed-stride and units kernels keep everything in registers (round 6:
    one extra per-lane counter made the SSTable walks spill 12-20 bytes to
    scratch, and SSTable verify / trailer CRCs / seal lost 1.3-2.5 points of
    HBM peak against round 5's build on the same box, profiles/r06/events_ab/).
    A scratch access in the round loop sits in the same in-order vmcnt queue as
    the row loads."""
    src = os.path.join(REPO, "lsbm_amd", "csrc", "crc32c_kernels.hip")
    s_file = tmp_path / "crc32c_kernels.s"
    subprocess.run([HIPCC if os.path.exists(HIPCC) else "hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    "-w", "-I", os.path.join(REPO, "include"), "-mllvm", "-amdgpu-atomic-optimizer-strategy=None",
                    "--cuda-device-only", "-S", "-o", str(s_file), src], check=True, timeout=900)
    scratch, name = {}, None
    for line in s_file.read_text().splitlines():
        m = re.match(r"^(_Z\w+):", line)
        if m:
            name = m.group(1)
        m = re.match(r"^; ScratchSize: (\d+)", line)
        if m and name:
            scratch[name] = int(m.group(1))
    crc = {k: v for k, v in scratch.items() if "crc32c_fixed_kernel" in k or "crc32c_units_kernel" in k}
    assert len(crc) >= 10, sorted(scratch)
    assert not {k: v for k, v in crc.items() if v}, crc
