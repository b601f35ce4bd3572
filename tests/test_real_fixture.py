"""Parity against bytes written by the reference itself (tests/golden/real_*):
SSTable blocks sealed by lsbm's TableBuilder::WriteRawBlock and WAL records
sealed by log::Writer::EmitPhysicalRecord, produced by the reference db_bench
(tests/golden/make_real_fixture.py).  CPU tests pin the oracle and the scalar
API; GPU tests run the batched seal / verify / WAL paths through the C ABI."""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def real():
    meta = json.load(open(os.path.join(G, "real_fixture.json")))
    sst = np.fromfile(os.path.join(G, "real_sst.bin"), dtype=np.uint8)
    wal = np.fromfile(os.path.join(G, "real_wal.bin"), dtype=np.uint8)
    return meta, sst, wal


def test_oracle_reproduces_reference_sst_trailers(oracle, real):
    meta, sst, _ = real
    assert len(meta["table_blocks"]) == 98
    for b in meta["table_blocks"]:
        o, n = b["offset"], b["size"]
        # ReadBlock: Unmask(DecodeFixed32(data + n + 1)) == Value(data, n + 1)
        assert oracle.unmask(b["stored_masked_crc"]) == oracle.value(sst[o:o + n + 1].tobytes())
        # WriteRawBlock: Mask(Extend(Value(block), &type, 1))
        crc = oracle.extend(oracle.value(sst[o:o + n].tobytes()), bytes([b["type"]]))
        assert oracle.mask(crc) == b["stored_masked_crc"]


def test_oracle_reproduces_reference_wal_records(oracle, real):
    meta, _, wal = real
    for r in meta["wal_records"]:
        o, n, t = r["offset"], r["length"], r["type"]
        type_crc = oracle.value(bytes([t]))  # log::Writer type_crc_ (common/log_writer.cc:18-21)
        crc = oracle.extend(type_crc, wal[o + 7:o + 7 + n].tobytes())
        assert oracle.mask(crc) == r["stored_masked_crc"]
        # log::Reader: Value(header + 6, 1 + length) (common/log_reader.cc:230-231)
        assert oracle.value(wal[o + 6:o + 7 + n].tobytes()) == oracle.unmask(r["stored_masked_crc"])


def test_scalar_api_on_reference_output(product_lib, real):
    from lsbm_amd import crc32c
    meta, sst, wal = real
    for b in meta["table_blocks"]:
        o, n = b["offset"], b["size"]
        assert crc32c.unmask(b["stored_masked_crc"]) == crc32c.value(sst[o:o + n + 1].tobytes())
    for r in meta["wal_records"]:
        o, n, t = r["offset"], r["length"], r["type"]
        assert crc32c.mask(crc32c.extend(crc32c.value(bytes([t])), wal[o + 7:o + 7 + n].tobytes())) \
            == r["stored_masked_crc"]


@pytest.mark.gpu
def test_gpu_verify_and_reseal_reference_sstable(torch_cuda, real):
    torch = torch_cuda
    from lsbm_amd import table
    meta, sst, _ = real
    handles = np.array([[b["offset"], b["size"]] for b in meta["table_blocks"]],
                       dtype=np.int64).reshape(-1)
    img = torch.from_numpy(sst.copy()).to("cuda")
    dh = torch.from_numpy(handles).to("cuda")
    st, ok = table.verify_status(img, dh)
    assert st.ok() and bool(ok.all())
    # wipe every trailer and re-seal: must reproduce the reference's bytes
    wiped = sst.copy()
    types = np.array([b["type"] for b in meta["table_blocks"]], dtype=np.uint8)
    for b in meta["table_blocks"]:
        wiped[b["offset"] + b["size"]:b["offset"] + b["size"] + 5] = 0
    img2 = torch.from_numpy(wiped).to("cuda")
    table.seal_blocks(img2, dh, torch.from_numpy(types).to("cuda"))
    assert np.array_equal(img2.cpu().numpy(), sst)
    # one flipped bit in a data block -> exactly that block fails
    img[meta["table_blocks"][10]["offset"] + 77] ^= 0x04
    st, ok = table.verify_status(img, dh)
    assert st.IsCorruption() and np.nonzero(ok.cpu().numpy() == 0)[0].tolist() == [10]


@pytest.mark.gpu
def test_gpu_wal_records_with_type_crc_init(torch_cuda, oracle, real):
    """Batched log::Writer seal, crc = Mask(Extend(type_crc_[t], payload, n))
    (common/log_writer.cc:86-87), and the log::Reader check, Value over
    [type || payload] (common/log_reader.cc:230-231), on the reference's WAL."""
    torch = torch_cuda
    from lsbm_amd import engine
    meta, _, wal = real
    recs = meta["wal_records"]
    d = torch.from_numpy(wal.copy()).to("cuda")
    payload = np.array([[r["offset"] + 7, r["length"]] for r in recs], dtype=np.int64).reshape(-1)
    init = np.array([oracle.value(bytes([r["type"]])) for r in recs], dtype=np.uint32)
    got = engine.crc32c_extents(d, torch.from_numpy(payload).to("cuda"),
                                init=torch.from_numpy(init.view(np.int32)).to("cuda"), masked=True)
    want = np.array([r["stored_masked_crc"] for r in recs], dtype=np.uint32)
    assert np.array_equal(got.cpu().numpy().view(np.uint32), want)
    reader = np.array([[r["offset"] + 6, r["length"] + 1] for r in recs], dtype=np.int64).reshape(-1)
    got2 = engine.crc32c_extents(d, torch.from_numpy(reader).to("cuda"))
    assert np.array_equal(got2.cpu().numpy().view(np.uint32),
                          np.array([oracle.unmask(int(x)) for x in want], dtype=np.uint32))
