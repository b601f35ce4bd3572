"""Snappy block codec: oracle pinning (CPU) and GPU parity (`-m gpu`).

The reference compresses SSTable blocks through port::Snappy_* (port/port_posix.h:119-150
-> libsnappy RawCompress / GetUncompressedLength / RawUncompress), from
TableBuilder::WriteBlock (table/table_builder.cc:181-193: keep the compressed form
only if it saves at least 1/8) and ReadBlock (table/format.cc:124-141:
"corrupted compressed block contents" when either call fails).  libsnappy is a
third-party dependency absent from /root/reference; the oracle
(oracle/snappy_oracle.c) is pinned to the libsnappy inside pyarrow through
tests/golden/snappy_fixture.json (tests/golden/make_snappy_fixture.py).
"""
import hashlib
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
from snappy_inputs import block, varint32  # noqa: E402


def sha(b):
    return hashlib.sha256(b).hexdigest()


def crafted_bytes(name, rec):
    if rec["hex"] is not None:
        return bytes.fromhex(rec["hex"])
    assert name == "literal_ext3"
    return varint32(70000) + bytes([62 << 2]) + (69999).to_bytes(3, "little") + b"z" * 70000


# ---------------------------------------------------------------- oracle pinning (CPU)

def test_oracle_compress_matches_libsnappy(snappy_oracle, snappy_golden):
    for cs in snappy_golden["cases"]:
        d = block(cs["kind"], cs["n"], cs["seed"])
        c = snappy_oracle.compress(d)
        assert len(c) == cs["clen"] and sha(c) == cs["csha"], (cs["kind"], cs["n"])
        assert c[:24].hex() == cs["head"]
        assert (len(c) < cs["n"] - cs["n"] // 8) == cs["store_compressed"]
        assert snappy_oracle.uncompress(c) == (True, d)


def test_oracle_uncompress_corruptions_match_libsnappy(snappy_oracle, snappy_golden):
    from make_snappy_fixture import mutations
    cases = snappy_golden["cases"]
    by_case = {}
    for rec in snappy_golden["corrupt"]:
        by_case.setdefault(rec["case"], []).append(rec)
    n_ok = 0
    for i, recs in by_case.items():
        cs = cases[i]
        c = snappy_oracle.compress(block(cs["kind"], cs["n"], cs["seed"]))
        muts = dict(mutations(c, 7000 + i))
        for rec in recs:
            ok, out = snappy_oracle.uncompress(muts[rec["mutation"]])
            assert ok == rec["ok"], (i, rec["mutation"])
            if ok:
                n_ok += 1
                assert len(out) == rec["out_len"] and sha(out) == rec["out_sha"]
    assert 0 < n_ok < len(snappy_golden["corrupt"])


def test_oracle_crafted_streams_match_libsnappy(snappy_oracle, snappy_golden):
    for rec in snappy_golden["crafted"]:
        ok, out = snappy_oracle.uncompress(crafted_bytes(rec["name"], rec))
        assert ok == rec["ok"], rec["name"]
        if ok:
            assert len(out) == rec["out_len"] and sha(out) == rec["out_sha"], rec["name"]


def test_oracle_length_and_bounds(snappy_oracle):
    assert snappy_oracle.max_compressed_length(4096) == 32 + 4096 + 4096 // 6
    assert snappy_oracle.uncompressed_length(varint32(300)) == (True, 300)
    assert snappy_oracle.uncompressed_length(b"") == (False, 0)
    assert snappy_oracle.uncompressed_length(bytes([0xFF, 0xFF, 0xFF, 0xFF, 0x0F])) == (True, 0xFFFFFFFF)
    # a capacity below the preamble length fails, like an undersized output buffer
    c = snappy_oracle.compress(b"abc" * 100)
    assert snappy_oracle.uncompress(c, cap=299) == (False, b"")
