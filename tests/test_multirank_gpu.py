"""bench.py's N > 1 path on the one-GPU box: `python bench.py --gpus 2` starts
its own two ranks (torch.distributed.run as a child process), each rank
checksums its own config-5 shard on the HIP path: global blocks [10M r,
10M (r + 1)) of the one 80M x 4 KiB dataset (BASELINE.json configs[4]; block i
= bytes [4096 i, 4096 (i + 1)) of the splitmix64 stream 0x5EED0000), and the
per-rank results are checked here against the oracle by global block index.
Both ranks share the one MI355X (LSBM_BENCH_DEVICES=1) and meet over bench.py's
DEFAULT backend (gloo on CPU tensors for the barrier and the MAX of the elapsed
time: no RCCL anywhere), the same code the driver's 8-GPU run executes."""
import glob
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from golden.splitmix import stream_bytes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_launches_two_ranks_config5_shards(torch_cuda, oracle, tmp_path):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
                        "LSBM_BENCH_BACKEND")}
    env.update(LSBM_BENCH_DEVICES="1")
    prefix = str(tmp_path / "samples")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
                        "--dump-samples", prefix],
                       env=env, capture_output=True, text=True, timeout=600, cwd=REPO)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["config"]["blocks_per_gpu"] == 10_000_000
    assert "over gloo" in line["config"]["parallelism"]  # the default: no RCCL in the harness
    # the per-rank table: both ranks, their bytes add up to the aggregate, and
    # the slowest rank's time is the reported one (MAX over ranks)
    rk = line["ranks"]
    assert [r["rank"] for r in rk] == [0, 1]
    total = sum(r["bytes"] for r in rk)
    assert total == 2 * 10_000_000 * 4096 * line["steps"]
    t_max = max(r["elapsed_s"] for r in rk)
    assert abs(total / t_max / 2**30 - line["value"]) <= 0.01 * line["value"]
    assert all(r["device"] == 0 and r["GiBps"] > 0 and r["kernel_ms_per_launch"] > 0 for r in rk)
    files = sorted(glob.glob(prefix + ".rank*.npz"))
    assert len(files) == 2
    seen = []
    for f in files:
        z = np.load(f)
        assert int(z["world"]) == 2 and int(z["n"]) == 10_000_000
        assert int(z["seed"]) == 0x5EED0000  # one dataset for every rank
        rank = int(f.rsplit(".rank", 1)[1].split(".")[0])
        g = z["gidx"].astype(np.int64)
        assert g.min() >= rank * 10_000_000 and g.max() < (rank + 1) * 10_000_000
        for i, c in zip(g, z["crc"]):
            assert c == oracle.value(stream_bytes(0x5EED0000, int(i) * 4096, 4096).tobytes()), (f, int(i))
        # every CRC of the shard at once, by linearity (10M blocks: n even)
        assert int(z["xor_crc"][0]) == oracle.value(z["xor_block"].tobytes()) ^ oracle.value(bytes(4096)), f
        seen.append((g.min(), g.max()))
    # rank 1's first block is global block 10M: the shards tile the dataset
    assert sorted(seen)[1][0] == 10_000_000


def test_bench_rejects_world_size_mismatch():
    """WORLD_SIZE set by a launcher but != --gpus is an error, not a warning
    (exits before any GPU call, so this runs on CPU)."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 2
    assert "WORLD_SIZE" in r.stderr
