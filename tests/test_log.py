"""WAL / MANIFEST records (common/log_writer.cc, common/log_reader.cc of lsbm).

Parity is pinned by tests/golden/log_fixture.json, which the reference's own
log::Writer and log::Reader produced (tests/golden/make_log_fixture.py):
  * the writer's image (length, crc32c, every header's CRC bytes);
  * for 25 corruption scenarios, the reader's exact output: each record
    (length, crc32c, LastRecordOffset) and each Reporter::Corruption call.
CPU tests: the fixture against the oracle, and BatchWriter's framing (no CRC).
GPU tests: BatchWriter::Seal, BatchReader (include/lsbm/log_checksum.h) and
the lsbm_log_seal_dev / lsbm_log_verify_dev entry points.
"""
import json
import os
import subprocess

import numpy as np
import pytest

from golden.splitmix import printable_bytes, stream_bytes

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def fx():
    with open(os.path.join(HERE, "golden", "log_fixture.json")) as f:
        d = json.load(f)
    lens = d["lens"]
    payload = printable_bytes(d["seed"], int(sum(lens)))
    offs = np.zeros(len(lens) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    return d, payload, offs


@pytest.fixture(scope="module")
def log_tool(product_lib, tmp_path_factory):
    exe = tmp_path_factory.mktemp("logtool") / "log_tool"
    libdir = os.path.join(REPO, "lsbm_amd")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(REPO, "include"),
                    os.path.join(HERE, "cpp", "log_tool.cc"), "-L", libdir, "-llsbm_crc32c",
                    "-Wl,-rpath," + libdir, "-o", str(exe)], check=True)
    return str(exe)


def _files(tmp_path, payload, offs):
    p, o = tmp_path / "payload.bin", tmp_path / "offs.bin"
    payload.tofile(p)
    offs.astype("<u8").tofile(o)
    return str(p), str(o)


def _apply(img, ops):
    img = img.copy()
    for op in ops:
        if op[0] == "xor":
            img[op[1]] ^= op[2]
        elif op[0] == "set":
            b = np.frombuffer(bytes.fromhex(op[2]), np.uint8)
            img[op[1]:op[1] + b.size] = b
        elif op[0] == "zero":
            img[op[1]:op[1] + op[2]] = 0
        elif op[0] == "truncate":
            img = img[:op[1]]
    return img


def _reference_image(d, layout, heads):
    """The reference writer's image: our layout + the fixture's header CRCs."""
    img = layout.copy()
    for h, c in zip(heads, d["image"]["header_crcs"]):
        img[h:h + 4] = np.frombuffer(bytes.fromhex(c), np.uint8)
    return img


# ---------------------------------------------------------------- CPU
def test_fixture_events_match_oracle(fx, oracle):
    """The clean scenario's records are the payloads, with the oracle's CRCs."""
    d, payload, offs = fx
    clean = [s for s in d["scenarios"] if s["name"] == "clean"][0]["events"].splitlines()
    assert len(clean) == len(d["lens"])
    for i, line in enumerate(clean):
        tag, n, crc, _ = line.split()
        rec = payload[int(offs[i]):int(offs[i + 1])].tobytes()
        assert tag == "R" and int(n) == len(rec) and int(crc, 16) == oracle.value(rec)


def test_batch_writer_framing_matches_reference(fx, log_tool, oracle, tmp_path):
    """BatchWriter::AddRecord lays out the reference writer's bytes exactly
    (CRC fields aside); host-only, no device needed."""
    d, payload, offs = fx
    p, o = _files(tmp_path, payload, offs)
    out = tmp_path / "layout.bin"
    r = subprocess.run([log_tool, "layout", p, o, str(out)], capture_output=True, text=True,
                       check=True)
    heads = [int(x) for x in r.stdout.split()]
    layout = np.fromfile(out, dtype=np.uint8)
    assert len(heads) == len(d["image"]["header_crcs"])
    assert layout.size == d["image"]["bytes"]
    assert all(layout[h:h + 4].tobytes() == bytes(4) for h in heads)
    img = _reference_image(d, layout, heads)
    assert oracle.value(img.tobytes()) == d["image"]["crc32c"]
    # the Python framing helper agrees
    from lsbm_amd import log
    img2, heads2 = log.layout_records(payload[int(offs[i]):int(offs[i + 1])]
                                      for i in range(len(d["lens"])))
    assert np.array_equal(img2, layout) and heads2.tolist() == heads


def test_reference_header_crcs_satisfy_reader_check(fx, log_tool, oracle, tmp_path):
    """Every reference header: Unmask(crc) == Value(header + 6, 1 + length)."""
    d, payload, offs = fx
    p, o = _files(tmp_path, payload, offs)
    out = tmp_path / "layout.bin"
    r = subprocess.run([log_tool, "layout", p, o, str(out)], capture_output=True, text=True,
                       check=True)
    heads = [int(x) for x in r.stdout.split()]
    img = _reference_image(d, np.fromfile(out, dtype=np.uint8), heads)
    for h in heads:
        length = int(img[h + 4]) | int(img[h + 5]) << 8
        stored = int.from_bytes(img[h:h + 4].tobytes(), "little")
        assert oracle.unmask(stored) == oracle.value(img[h + 6:h + 7 + length].tobytes())


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 37, 0])
def test_batch_writer_seal_reproduces_reference_image(torch_cuda, fx, log_tool, oracle, tmp_path,
                                                      batch):
    """Group commits of `batch` records (0: one Seal at the end) give the
    reference writer's image byte for byte."""
    d, payload, offs = fx
    p, o = _files(tmp_path, payload, offs)
    out = tmp_path / "sealed.bin"
    subprocess.run([log_tool, "write", p, o, str(out), str(batch)], check=True,
                   capture_output=True, timeout=120)
    img = np.fromfile(out, dtype=np.uint8)
    assert img.size == d["image"]["bytes"]
    assert oracle.value(img.tobytes()) == d["image"]["crc32c"]


@pytest.mark.gpu
def test_batch_reader_matches_reference_reader(torch_cuda, fx, log_tool, tmp_path):
    """BatchReader: same records, offsets and Reporter calls as the
    reference's log::Reader on every corruption scenario of the fixture."""
    d, payload, offs = fx
    p, o = _files(tmp_path, payload, offs)
    out = tmp_path / "layout.bin"
    r = subprocess.run([log_tool, "layout", p, o, str(out)], capture_output=True, text=True,
                       check=True)
    heads = [int(x) for x in r.stdout.split()]
    base = _reference_image(d, np.fromfile(out, dtype=np.uint8), heads)
    failed = []
    for s in d["scenarios"]:
        img = _apply(base, s["ops"])
        path = tmp_path / f"{s['name']}.bin"
        img.tofile(path)
        got = subprocess.run([log_tool, "read", str(path)], capture_output=True, text=True,
                             check=True, timeout=120).stdout
        if got != s["events"]:
            failed.append(s["name"])
    assert not failed, failed


@pytest.mark.gpu
def test_batch_reader_initial_offset_matches_reference_reader(torch_cuda, fx, log_tool, tmp_path):
    """BatchReader with initial_offset != 0: SkipToInitialBlock, records that
    start before the offset skipped, drops before it unreported -- the same
    events as the reference's log::Reader (common/log_reader.cc:35-57,
    171-176, 247-251) on every initial-offset scenario of the fixture."""
    d, payload, offs = fx
    p, o = _files(tmp_path, payload, offs)
    out = tmp_path / "layout.bin"
    r = subprocess.run([log_tool, "layout", p, o, str(out)], capture_output=True, text=True,
                       check=True)
    heads = [int(x) for x in r.stdout.split()]
    base = _reference_image(d, np.fromfile(out, dtype=np.uint8), heads)
    assert len(d["offset_scenarios"]) >= 20
    failed = []
    for s in d["offset_scenarios"]:
        img = _apply(base, s["ops"])
        path = tmp_path / f"off_{s['name']}.bin"
        img.tofile(path)
        got = subprocess.run([log_tool, "read", str(path), str(s["initial_offset"])],
                             capture_output=True, text=True, check=True, timeout=120).stdout
        if got != s["events"]:
            failed.append(s["name"])
    assert not failed, failed


@pytest.mark.gpu
def test_log_seal_and_verify_entry_points(torch_cuda, oracle):
    """lsbm_log_seal_dev / lsbm_log_verify_dev on a framed image: seals equal
    Mask(Extend(type_crc_[t], payload)) (common/log_writer.cc:86-87), verify
    flags exactly the flipped records, headers outside the image are bad."""
    torch = torch_cuda
    from lsbm_amd import log
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 5000, size=3000)
    lens[::97] = rng.integers(30000, 80000, size=lens[::97].size)  # fragmented records
    payloads = [stream_bytes(int(i) + 11, 0, int(n)).tobytes() for i, n in enumerate(lens)]
    img, heads = log.layout_records(payloads)
    d = torch.from_numpy(img).to("cuda")
    dh = torch.from_numpy(heads).to("cuda")
    masked, nbad = log.seal_records(d, dh)
    sealed = d.cpu().numpy()
    assert int(nbad.item()) == 0
    got = masked.cpu().numpy().view(np.uint32)
    for i in rng.choice(heads.size, size=300, replace=False):
        h = int(heads[i])
        n, t = int(sealed[h + 4]) | int(sealed[h + 5]) << 8, int(sealed[h + 6])
        want = oracle.mask(oracle.extend(oracle.value(bytes([t])), sealed[h + 7:h + 7 + n].tobytes()))
        assert got[i] == want
        assert int.from_bytes(sealed[h:h + 4].tobytes(), "little") == want
    ok, nbad = log.verify_records(d, dh)
    assert int(nbad.item()) == 0 and bool(ok.all())
    bad = sorted(int(i) for i in rng.choice(heads.size, size=40, replace=False))
    for i in bad:  # one bit of the payload, the type, or the stored crc
        h = int(heads[i])
        n = int(sealed[h + 4]) | int(sealed[h + 5]) << 8
        pos = h + int(rng.integers(0, 4)) if n == 0 else h + 7 + int(rng.integers(0, n))
        d[pos] ^= 1 << int(rng.integers(0, 8))
    ok, nbad = log.verify_records(d, dh)
    assert np.nonzero(ok.cpu().numpy() == 0)[0].tolist() == bad and int(nbad.item()) == len(bad)
    # headers past the end of the image, or whose payload runs past it
    h_last = int(heads[-1])
    short = d[:h_last + 8].clone()  # the last header + 1 payload byte
    last_len = int(sealed[h_last + 4]) | int(sealed[h_last + 5]) << 8
    fits = int(last_len <= 1)
    tail = torch.tensor([h_last + 8 - 3, h_last + 100, h_last], dtype=torch.int64, device="cuda")
    ok, nbad = log.verify_records(short, tail)
    assert ok.cpu().tolist() == [0, 0, fits] and int(nbad.item()) == 3 - fits
    _, nb2 = log.seal_records(short, tail)
    assert int(nb2.item()) == 3 - fits


def _log_crcs_oracle(oracle, img, heads, lens):
    """Mask(Value(type || payload)) of every record (common/log_writer.cc:85-88):
    the bytes [h + 6, h + 7 + len) are contiguous in the image."""
    parts = [img[int(h) + 6:int(h) + 7 + int(n)] for h, n in zip(heads, lens)]
    offs = np.zeros(len(parts) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([p.size for p in parts])
    buf = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return oracle.batch_offsets(buf, offs, masked=True)


@pytest.mark.gpu
@pytest.mark.parametrize("policy", [1, 2], ids=["units", "stream"])
@pytest.mark.parametrize("order", ["in_order", "shuffled"])
def test_log_seal_deferred_headers_past_the_image(torch_cuda, oracle, policy, order):
    """lsbm_log_seal_dev with d_masked (the stream kernel defers its header
    stores to each wave's end) on an image cut inside a record's payload near
    its end: records that fit get their header CRC written and in out[]; the
    cut record and every record after it (headers past the image) count as
    bad, get out[] = 0, and none of their bytes or the guard bytes after the
    image change.  Shuffled header offsets also send windows through the
    stream kernel's units fallback (the deferred path's bad-record
    branch was never run)."""
    torch = torch_cuda
    from lsbm_amd import log
    from lsbm_amd._lib import lib
    rng = np.random.default_rng(31 + policy)
    lens = rng.integers(0, 2541, size=12000)
    lens[-40] = 2000  # the record the cut lands in
    pay = stream_bytes(0xD1, 0, int(lens.sum()))
    po = np.concatenate([[0], np.cumsum(lens)])
    img, heads = log.layout_records(pay[po[i]:po[i + 1]].tobytes() for i in range(lens.size))
    plen = img[heads + 4].astype(np.int64) | (img[heads + 5].astype(np.int64) << 8)
    k = int(np.nonzero(plen > 100)[0][-5])  # a physical record near the end with a payload
    cut = int(heads[k]) + 7 + int(plen[k]) // 2
    guard = np.full(4096, 0xA5, dtype=np.uint8)
    full = np.concatenate([img[:cut], guard])
    before = full.copy()
    d_full = torch.from_numpy(full).to("cuda")
    d = d_full[:cut]
    idx = np.arange(heads.size)
    if order == "shuffled":
        rng.shuffle(idx)
    dh = torch.from_numpy(heads[idx].copy()).to("cuda")
    lib().lsbm_test_ragged_kernel(policy)
    try:
        masked, nbad = log.seal_records(d, dh)
        torch.cuda.synchronize()
    finally:
        lib().lsbm_test_ragged_kernel(0)
    out = d_full.cpu().numpy()
    got = masked.cpu().numpy().view(np.uint32)
    fits = heads[idx] + 7 + plen[idx] <= cut
    assert int(nbad.item()) == int((~fits).sum()) == heads.size - k
    assert np.array_equal(out[cut:], guard)
    want = _log_crcs_oracle(oracle, img, heads[idx][fits], plen[idx][fits])
    assert np.array_equal(got[fits], want)
    assert not got[~fits].any()
    hw = heads[idx][fits]
    stored = (out[hw].astype(np.uint32) | (out[hw + 1].astype(np.uint32) << 8) |
              (out[hw + 2].astype(np.uint32) << 16) | (out[hw + 3].astype(np.uint32) << 24))
    assert np.array_equal(stored, want)
    # nothing else changed: every byte but the fitting headers' CRC fields
    written = np.zeros(out.size, dtype=bool)
    for b in range(4):
        written[hw + b] = True
    assert np.array_equal(out[~written], before[~written])
