"""The drop-in claim, literally: the reference's own table/ (TableBuilder,
ReadBlock, the filter block), common/log_* and util/ code, compiled unchanged
from /root/reference, linked against lsbm_amd/liblsbm_crc32c.so instead of its
util/crc32c.cc and util/hash.cc, with this repo's include/ (util/crc32c.h,
util/hash.h) first on the include path (oracle/Makefile `reflink`).

tests/cpp/ref_table_link.cc writes a 20,000-entry SSTable with a bloom filter
block and a 3,000-record WAL, reads both back with checksums on, and reads a
copy with a flipped byte.  Both builds must write byte-identical files and
report the same results.  CPU only (the scalar API runs on the host); skipped
where /root/reference is absent (the GPU box)."""
import filecmp
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "table")), reason="needs /root/reference")
def test_reference_table_and_log_link_unchanged(tmp_path):
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(REPO, "oracle"), "reflink"], check=True)
    outs = {}
    for v in ("ref", "lsbm"):
        d = tmp_path / v
        d.mkdir()
        r = subprocess.run([os.path.join(REPO, "oracle", "_ref", "link_" + v), str(d)],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        # drop the reference's cache-statistics line (it carries a timestamp)
        outs[v] = [ln for ln in r.stdout.splitlines() if not ln.startswith("total:")]
    assert outs["ref"] == outs["lsbm"]
    got = "\n".join(outs["lsbm"])
    assert "table read (verify_checksums): OK entries 20000" in got
    assert "log read: records 3000 dropped 0" in got
    assert "corrupted table read: Corruption: block checksum mismatch" in got
    for f in ("000001.sst", "000002.log", "000003.sst"):
        assert filecmp.cmp(tmp_path / "ref" / f, tmp_path / "lsbm" / f, shallow=False), f
    # the lsbm build really takes Extend and Hash from the product library
    nm = subprocess.run(["nm", "-D", "--undefined-only",
                         os.path.join(REPO, "oracle", "_ref", "link_lsbm")],
                        capture_output=True, text=True).stdout
    assert "_ZN7leveldb6crc32c6ExtendEjPKcm" in nm and "_ZN7leveldb4HashEPKcmj" in nm


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "table")), reason="needs /root/reference")
def test_level2_binding_compiles_and_links_against_the_reference():
    """INTEGRATION.md's Level-2 binding is a real header
    (integration/leveldb_gpu_checksum.h): compiled with the reference's own
    flags and headers (leveldb::BlockHandle, Status, EncodeFixed32) and linked
    with its table/ and util/ objects, the library and the HIP runtime
    (oracle/Makefile gpubind).  tests/test_gpu_parity.py runs the binary."""
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(REPO, "oracle"), "gpubind"], check=True)
    exe = os.path.join(REPO, "oracle", "_ref", "gpu_binding")
    assert os.access(exe, os.X_OK)
    ldd = subprocess.run(["ldd", exe], capture_output=True, text=True).stdout
    assert "liblsbm_crc32c.so" in ldd and "libamdhip64" in ldd


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "table")), reason="needs /root/reference")
def test_gpu_table_builder_compiles_and_links_against_the_reference():
    """integration/gpu_table_builder.h (the reference's TableBuilder with its
    trailers reserved and sealed by one SealBlocks call per table) compiled
    with the reference's own headers and linked with its table/, util/ and
    common/ objects plus its own util/crc32c.cc and util/hash.cc (oracle/Makefile
    gputable): the unmodified TableBuilder in the binary takes Extend and Hash
    from the reference's sources, the GPU builder SealBlocks from the library.
    tests/test_gpu_parity.py runs it on the GPU."""
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(REPO, "oracle"), "gputable", "gpucompact"], check=True)
    assert os.access(os.path.join(REPO, "oracle", "_ref", "gpu_compaction"), os.X_OK)
    exe = os.path.join(REPO, "oracle", "_ref", "gpu_table_builder")
    assert os.access(exe, os.X_OK)
    syms = subprocess.run(["nm", exe], capture_output=True, text=True).stdout.splitlines()
    defined = {ln.split()[-1] for ln in syms if " T " in ln}
    undefined = {ln.split()[-1] for ln in syms if " U " in ln}
    assert "_ZN7leveldb6crc32c6ExtendEjPKcm" in defined  # the reference's own util/crc32c.cc
    assert "_ZN7leveldb4HashEPKcmj" in defined
    assert any("SealBlocks" in u for u in undefined)  # from liblsbm_crc32c.so
    ldd = subprocess.run(["ldd", exe], capture_output=True, text=True).stdout
    assert "liblsbm_crc32c.so" in ldd and "libamdhip64" in ldd


# config 1 (BASELINE.json configs[0]): lsbm's own db_bench write workload
# (SURVEY.md section 3.5), scaled by --writes
DB_BENCH_ARGS = ["--benchmarks=separate", "--write_workload=counter", "--value_size=100", "--write_key_from=0",
                 "--key_from=0", "--read_key_from=0", "--writespeed=-1", "--readspeed=0", "--random_reads=0",
                 "--read_threads=0", "--countdown=600", "--block_cache_size=0", "--histogram=0"]


def db_bench_args(db, writes):
    return [f"--db={db}", f"--writes={writes}", f"--write_key_upto={writes}", f"--key_upto={writes}",
            f"--read_key_upto={writes}"] + DB_BENCH_ARGS


def db_verify(exe, db, open_copy=None):
    """oracle/_ref/db_verify (reference code only) over a database directory:
    its JSON line, and with open_copy the DB::Open digest of a copy."""
    import json
    import shutil
    args = [exe, db]
    if open_copy:
        shutil.copytree(db, open_copy)
        args = [exe, open_copy, "--open"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=600)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    return r.returncode, json.loads(line)


def db_check_gpu(db, arg, tmp_path, *more):
    """tools/db_check_gpu.cc (this repo's layers only), built once per test, over
    a database directory: its JSON line."""
    import json
    exe = tmp_path / "db_check_gpu"
    if not exe.exists():
        lib = os.path.join(REPO, "lsbm_amd")
        subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", os.path.join(REPO, "include"),
                        os.path.join(REPO, "tools", "db_check_gpu.cc"), "-L", lib, "-llsbm_crc32c",
                        "-Wl,-rpath," + lib, "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), db, arg, *more], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "table")), reason="needs /root/reference")
def test_db_bench_builds_three_ways_and_level1_writes_the_same_database(tmp_path):
    """lsbm's db_bench from its own sources three ways (oracle/Makefile
    dbbench_gpu): as shipped; Level 1 (this repo's util/crc32c.h first, its
    Extend and Hash from liblsbm_crc32c.so); Level 2 (also
    integration/table_builder_gpu.cc in place of table/table_builder.o).  Here,
    without a GPU: the reference and the Level-1 build each run config 1 at
    200K writes, and the reference-only checker (tests/cpp/db_verify.cc) reads
    every block and log record of both databases with verification and finds
    the same database content (DB::Open digest).  tests/test_gpu_parity.py runs
    the Level-2 build on the GPU."""
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(REPO, "oracle"), "dbbench_gpu"], check=True)
    ref = os.path.join(REPO, "oracle", "_ref")
    syms = subprocess.run(["nm", os.path.join(ref, "db_bench_gpu")], capture_output=True, text=True).stdout
    assert " U _ZN7leveldb6crc32c6ExtendEjPKcm" in syms and " U _ZN7leveldb4HashEPKcmj" in syms
    assert any("SealBlocks" in ln and " U " in ln for ln in syms.splitlines())
    assert "_ZN7leveldb12TableBuilder6FinishEv" in syms
    ldd = subprocess.run(["ldd", os.path.join(ref, "db_bench_l1")], capture_output=True, text=True).stdout
    assert "liblsbm_crc32c.so" in ldd
    digests = {}
    for name in ("db_bench", "db_bench_l1"):
        db = tmp_path / name
        db.mkdir()
        r = subprocess.run([os.path.join(ref, name)] + db_bench_args(str(db), 200_000),
                           capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        assert "separate" in r.stdout
        rc, v = db_verify(os.path.join(ref, "db_verify"), str(db))
        assert rc == 0 and v["table_errors"] == 0 and v["log_errors"] == 0, v
        assert v["tables"] >= 1 and v["records"] > 0, v
        # tools/db_check_gpu.cc gathers the same blocks (its own footer / block parsing)
        g = db_check_gpu(str(db), "--parse-only", tmp_path)
        assert (g["tables"], g["unfinished"], g["blocks"]) == (v["tables"], v["unfinished"], v["blocks"]), (g, v)
        rc, v = db_verify(os.path.join(ref, "db_verify"), str(db), str(tmp_path / (name + "_open")))
        assert rc == 0 and v["open_error"] == "", v
        digests[name] = (v["live"], v["digest"])
    assert digests["db_bench"] == digests["db_bench_l1"]
