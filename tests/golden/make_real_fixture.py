"""Fixture of REAL reference output: SSTable blocks + trailers and WAL records
written by lsbm's own db_bench (oracle/_ref/db_bench, built from
/root/reference by `make -C oracle dbbench`).

    python tests/golden/make_real_fixture.py

Runs a 200k-put db_bench (the SURVEY.md 3.5 command, scaled down) into a temp
dir, then extracts
  * from one .ldb table: the first 96 data blocks, the metaindex block and the
    index block, each as [block n B][type 1 B][masked crc 4 B] exactly as
    TableBuilder::WriteRawBlock wrote them (table/table_builder.cc:237-255);
  * from the WAL: the first 200 physical records [crc 4][len 2][type 1][payload]
    as log::Writer::EmitPhysicalRecord wrote them (common/log_writer.cc:75-100).
  * the table's filter block (table/filter_block.cc format, written by
    InternalFilterPolicy over BloomFilterPolicy(20)): its filters up to the one
    that covers the last of those 96 data blocks, and the whole offset array.
Writes tests/golden/real_sst.bin, real_wal.bin, real_filter.bin and
real_fixture.json.  Only
bytes produced by the reference are stored; no reference source.
"""
import json
import os
import struct
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
DB_BENCH = os.path.join(REPO, "oracle", "_ref", "db_bench")
MAGIC = 0xDB4775248B80FB57  # table/format.h kTableMagicNumber


def varint(buf, pos):
    r, shift = 0, 0
    while True:
        b = buf[pos]
        pos += 1
        r |= (b & 0x7F) << shift
        if b < 0x80:
            return r, pos
        shift += 7


def handle(buf, pos):
    off, pos = varint(buf, pos)
    size, pos = varint(buf, pos)
    return (off, size), pos


def block_entries(block):
    """Decode a (block) -> [(key, value)] (table/block.cc format)."""
    n_restarts = struct.unpack_from("<I", block, len(block) - 4)[0]
    limit = len(block) - 4 - 4 * n_restarts
    pos, key, out = 0, b"", []
    while pos < limit:
        shared, pos = varint(block, pos)
        non_shared, pos = varint(block, pos)
        vlen, pos = varint(block, pos)
        key = key[:shared] + block[pos:pos + non_shared]
        pos += non_shared
        out.append((key, block[pos:pos + vlen]))
        pos += vlen
    return out


def main():
    if not os.path.exists(DB_BENCH):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "dbbench"], check=True)
    d = tempfile.mkdtemp(prefix="lsbm_db_")
    args = [DB_BENCH, f"--db={d}", "--benchmarks=separate", "--write_workload=counter",
            "--writes=200000", "--value_size=100", "--write_key_from=0",
            "--write_key_upto=200000", "--key_from=0", "--key_upto=200000",
            "--read_key_from=0", "--read_key_upto=200000", "--writespeed=-1", "--readspeed=0",
            "--random_reads=0", "--read_threads=0", "--countdown=30", "--block_cache_size=0",
            "--histogram=0"]
    subprocess.run(args, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, cwd=d)
    tables = sorted(f for f in os.listdir(d) if f.endswith(".ldb") or f.endswith(".sst"))
    logs = sorted(f for f in os.listdir(d) if f.endswith(".log"))
    tab = open(os.path.join(d, tables[0]), "rb").read()
    footer = tab[-48:]
    assert struct.unpack_from("<Q", footer, 40)[0] == MAGIC
    (meta_h, pos) = handle(footer, 0)
    (index_h, _) = handle(footer, pos)
    index_block = tab[index_h[0]:index_h[0] + index_h[1]]
    data_handles = [handle(v, 0)[0] for _, v in block_entries(index_block)]
    picked = [("data", h) for h in data_handles[:96]] + [("metaindex", meta_h),
                                                          ("index", index_h)]
    sst_bin, sst_meta = bytearray(), []
    for kind, (off, size) in picked:
        region = tab[off:off + size + 5]  # block || type || masked crc
        sst_meta.append({"kind": kind, "offset": len(sst_bin), "size": size,
                         "type": region[size],
                         "stored_masked_crc": struct.unpack_from("<I", region, size + 1)[0],
                         "file_offset": off})
        sst_bin += region
    meta_block = tab[meta_h[0]:meta_h[0] + meta_h[1]]
    filt = None
    for k, v in block_entries(meta_block):
        if k == b"filter.leveldb.BuiltinBloomFilter":  # table/table_builder.cc:280-284
            fh = handle(v, 0)[0]
            fb = tab[fh[0]:fh[0] + fh[1]]
            array_offset = struct.unpack_from("<I", fb, len(fb) - 5)[0]
            n_f = (len(fb) - 5 - array_offset) // 4
            offsets = list(struct.unpack_from("<%dI" % n_f, fb, array_offset))
            last = picked[95][1] if len(data_handles) > 95 else picked[-3][1]
            covered = (last[0] + last[1] + 5) // 2048  # filters complete after that block
            end = offsets[covered] if covered < n_f else array_offset
            filt = {"handle": list(fh), "base_lg": fb[-1], "array_offset": array_offset,
                    "offsets": offsets, "prefix_bytes": end}
            open(os.path.join(HERE, "real_filter.bin"), "wb").write(fb[:end])
    wal = open(os.path.join(d, logs[0]), "rb").read()
    wal_bin, wal_meta, pos = bytearray(), [], 0
    while len(wal_meta) < 200 and pos + 7 <= len(wal):
        block_left = 32768 - (pos % 32768)  # common/log_format.h kBlockSize
        if block_left < 7:
            pos += block_left  # trailer padding
            continue
        crc, length, typ = struct.unpack_from("<IHB", wal, pos)
        if typ == 0 and length == 0:
            break
        rec = wal[pos:pos + 7 + length]
        wal_meta.append({"offset": len(wal_bin), "length": length, "type": typ,
                         "stored_masked_crc": crc})
        wal_bin += rec
        pos += 7 + length
    open(os.path.join(HERE, "real_sst.bin"), "wb").write(sst_bin)
    open(os.path.join(HERE, "real_wal.bin"), "wb").write(wal_bin)
    json.dump({"source": "lsbm db_bench built from /root/reference (oracle/Makefile dbbench); "
                         + " ".join(os.path.basename(a) if i == 0 else a
                                    for i, a in enumerate(args) if not a.startswith("--db=")),
               "table_file": tables[0], "table_blocks": sst_meta, "filter": filt,
               "wal_file": logs[0], "wal_records": wal_meta},
              open(os.path.join(HERE, "real_fixture.json"), "w"), indent=0)
    print(f"{len(sst_meta)} table blocks ({len(sst_bin)} B), {len(wal_meta)} WAL records "
          f"({len(wal_bin)} B)")


if __name__ == "__main__":
    sys.exit(main())
