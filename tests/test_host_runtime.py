"""CPU checks of the host runtime under the C++ layers (no GPU compute).

* NUMA placement inputs: a GPU's PCI bus id -> <sysfs>/bus/pci/devices/<id>/
  numa_node (host_numa.cc), cpulist parsing, the cgroup CPU quota (v2 cpu.max
  and v1 cfs files), all against fake sysfs / cgroup trees;
* the worker pool: sized from the usable cores (affinity mask capped by the
  cgroup quota), and jobs of concurrent callers run at the same time instead
  of taking turns for the whole pool (round 3's pool ran one job at a time).

SURVEY.md 8(e) asks for each GPU's shard to be staged from pinned memory on
that GPU's NUMA node; the reference's writer, compaction and reader threads
run concurrently (util/env_posix.cc:546-586, lsbm/db_bench.cc:711-736).
"""
import ctypes
import os

import pytest


def _lib(product_lib):
    from lsbm_amd import _lib
    return _lib.lib()


def test_pci_bus_id_to_numa_node(product_lib, tmp_path):
    lib = _lib(product_lib)
    devs = tmp_path / "bus" / "pci" / "devices"
    for bdf, node in (("0000:0a:00.0", "0\n"), ("0000:8b:00.0", "1\n"), ("0000:c1:00.0", "-1\n"),
                      ("0000:d9:00.0", "garbage\n")):
        (devs / bdf).mkdir(parents=True)
        (devs / bdf / "numa_node").write_text(node)
    root = str(tmp_path).encode()
    assert lib.lsbm_test_pci_numa_node(root, b"0000:0a:00.0") == 0
    assert lib.lsbm_test_pci_numa_node(root, b"0000:8B:00.0") == 1  # (HIP may report upper case)
    assert lib.lsbm_test_pci_numa_node(root, b"0000:c1:00.0") == -1  # no NUMA information
    assert lib.lsbm_test_pci_numa_node(root, b"0000:d9:00.0") == -1
    assert lib.lsbm_test_pci_numa_node(root, b"0000:ff:00.0") == -1  # absent
    assert lib.lsbm_test_pci_numa_node(root, b"") == -1


@pytest.mark.parametrize("text,want", [
    ("0-3,8,10-11", [0, 1, 2, 3, 8, 10, 11]),
    ("0-63,128-191\n", list(range(64)) + list(range(128, 192))),
    ("5", [5]),
    ("", []),
    ("\n", []),
    ("3-1", None),
    ("a-b", None),
    ("1,,2", [1, 2]),
    ("0-", None),
])
def test_cpulist_parsing(product_lib, text, want):
    lib = _lib(product_lib)
    buf = (ctypes.c_int * 512)()
    n = lib.lsbm_test_parse_cpulist(text.encode(), buf, 512)
    if want is None:
        assert n == -1
    else:
        assert n == len(want) and list(buf[:n]) == want


def test_cgroup_quota(product_lib, tmp_path):
    lib = _lib(product_lib)
    v2 = tmp_path / "v2"
    v2.mkdir()
    (v2 / "cpu.max").write_text("1600000 100000\n")  # the GPU box: 16 CPUs
    assert lib.lsbm_test_cgroup_quota(str(v2).encode()) == 16
    (v2 / "cpu.max").write_text("max 100000\n")
    assert lib.lsbm_test_cgroup_quota(str(v2).encode()) == 0
    (v2 / "cpu.max").write_text("50000 100000\n")  # half a CPU still counts as one
    assert lib.lsbm_test_cgroup_quota(str(v2).encode()) == 1
    v1 = tmp_path / "v1" / "cpu"
    v1.mkdir(parents=True)
    (v1 / "cpu.cfs_quota_us").write_text("250000\n")
    (v1 / "cpu.cfs_period_us").write_text("100000\n")
    assert lib.lsbm_test_cgroup_quota(str(tmp_path / "v1").encode()) == 2
    (v1 / "cpu.cfs_quota_us").write_text("-1\n")
    assert lib.lsbm_test_cgroup_quota(str(tmp_path / "v1").encode()) == 0
    assert lib.lsbm_test_cgroup_quota(str(tmp_path / "none").encode()) == 0


def test_pool_sized_from_usable_cores(product_lib):
    lib = _lib(product_lib)
    usable = len(os.sched_getaffinity(0))
    q = lib.lsbm_test_cgroup_quota(None)
    if q > 0:
        usable = min(usable, q)
    if os.environ.get("LSBM_HOST_THREADS"):
        usable = int(os.environ["LSBM_HOST_THREADS"])
    assert lib.lsbm_host_threads() == max(1, usable - 1)


def test_pool_runs_concurrent_callers_at_once(product_lib):
    """4 callers x 6 jobs of 2 pieces (3 ms each) against 1 caller x 24 of the
    same jobs: the pool serves the callers' jobs side by side (at least two
    jobs have pieces running at the same moment) and the work finishes
    measurably sooner than one job at a time."""
    lib = _lib(product_lib)
    if lib.lsbm_host_threads() < 3:
        pytest.skip("needs >= 3 pool threads")
    t_serial, t_conc = ctypes.c_double(), ctypes.c_double()
    peak1 = lib.lsbm_test_pool_overlap(1, 24, 2, 3000, ctypes.byref(t_serial))
    peak4 = lib.lsbm_test_pool_overlap(4, 6, 2, 3000, ctypes.byref(t_conc))
    assert peak1 == 1
    assert peak4 >= 2
    assert t_conc.value < 0.8 * t_serial.value, (t_conc.value, t_serial.value)


def test_pool_nested_jobs_and_errors(product_lib):
    lib = _lib(product_lib)
    assert lib.lsbm_test_pool_overlap(0, 1, 1, 0, None) == -1
    assert lib.lsbm_test_pool_overlap(2, 3, 1, 0, None) >= 0  # one-piece jobs run inline
    assert lib.lsbm_test_pool_overlap(8, 4, 64, 50, None) >= 1


def test_pool_every_piece_runs_once_under_contention(product_lib):
    """The lock-free pool (job slots taken under hazard pointers, pieces
    claimed by fetch_add): 8 callers x 400 jobs of 1-64 pieces, a fifth of
    them running nested jobs inside their pieces -- more jobs at once than the
    pool has threads -- and every piece of every job runs exactly once; then
    more callers than the 64 job slots (the overflow runs inline)."""
    lib = _lib(product_lib)
    lib.lsbm_test_pool_stress.argtypes = [ctypes.c_int] * 3
    assert lib.lsbm_test_pool_stress(0, 1, 1) == -1
    assert lib.lsbm_test_pool_stress(8, 400, 64) == 0
    assert lib.lsbm_test_pool_stress(80, 20, 16) == 0


def test_pool_under_thread_sanitizer(tmp_path):
    """The same stress, built with -fsanitize=thread (host code only): no data
    race reported, every piece once (tests/cpp/pool_tsan.cc)."""
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    csrc = os.path.join(repo, "lsbm_amd", "csrc")
    exe = tmp_path / "pool_tsan"
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-D__HIP_PLATFORM_AMD__",
                        "-I", os.path.join(repo, "include"), "-I", "/opt/rocm/include",
                        os.path.join(repo, "tests", "cpp", "pool_tsan.cc"), os.path.join(csrc, "host_session.cc"),
                        os.path.join(csrc, "host_numa.cc"), os.path.join(csrc, "status.cc"),
                        "-L", "/opt/rocm/lib", "-lamdhip64", "-lpthread", "-Wl,-rpath,/opt/rocm/lib",
                        "-o", str(exe)], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("no ThreadSanitizer build here: " + r.stderr[-300:])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert r.stdout.startswith("OK"), r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-3000:]


def test_cgroup_quota_of_the_process_own_cgroup(product_lib, tmp_path):
    """usable_cores() reads the quota of the process's OWN cgroup (its path in
    /proc/self/cgroup), the smallest over it and its ancestors -- not the
    mount root's, which has no cpu.max without a cgroup namespace (ADVICE r4:
    a box with 256 CPUs and a 16-CPU quota would otherwise size ~255 workers)."""
    lib = _lib(product_lib)
    root = tmp_path / "cg"
    leaf = root / "kubepods" / "pod1" / "ctr"
    leaf.mkdir(parents=True)
    (root / "kubepods" / "cpu.max").write_text("max 100000\n")
    (root / "kubepods" / "pod1" / "cpu.max").write_text("3200000 100000\n")  # 32 CPUs
    (leaf / "cpu.max").write_text("1600000 100000\n")  # 16 CPUs
    r = str(root).encode()
    assert lib.lsbm_test_cgroup_quota(r) == 0  # the mount root alone: no quota
    assert lib.lsbm_test_cgroup_quota_of(r, b"0::/kubepods/pod1/ctr\n") == 16
    (leaf / "cpu.max").write_text("max 100000\n")  # the parent's limit binds the child
    assert lib.lsbm_test_cgroup_quota_of(r, b"0::/kubepods/pod1/ctr\n") == 32
    assert lib.lsbm_test_cgroup_quota_of(r, b"0::/kubepods/pod1/ctr/\n") == 32
    # a cgroup namespace shows "/": the mount root is the process's cgroup
    (root / "cpu.max").write_text("800000 100000\n")
    assert lib.lsbm_test_cgroup_quota_of(r, b"0::/\n") == 8
    assert lib.lsbm_test_cgroup_quota_of(r, b"0::/nowhere\n") == 8  # nothing on the path: the root's
    # cgroup v1 (hybrid hosts, like this container): the line whose controllers include cpu
    v1 = tmp_path / "v1"
    d = v1 / "cpu,cpuacct" / "jobs" / "j7"
    d.mkdir(parents=True)
    (d / "cpu.cfs_quota_us").write_text("400000\n")
    (d / "cpu.cfs_period_us").write_text("100000\n")
    text = b"9:name=systemd:/\n4:memory:/x\n2:cpuacct,cpu:/jobs/j7\n0::/\n"
    assert lib.lsbm_test_cgroup_quota_of(str(v1).encode(), text) == 4
    assert lib.lsbm_test_cgroup_quota_of(str(v1).encode(), b"3:cpuset:/jobs/j7\n") == 0  # not cpu
    assert lib.lsbm_test_cgroup_quota_of(str(v1).encode(), b"") == 0
    assert lib.lsbm_test_cgroup_quota_of(str(v1).encode(), b"garbage") == 0


def test_pool_job_helper_cap(product_lib):
    """A job takes at most max_helpers pool workers besides its caller: the
    staging copies use copy_helpers() (3 by default: one thread already copies
    ~50 GB/s and PCIe takes ~56), not every core of the quota."""
    lib = _lib(product_lib)
    if lib.lsbm_host_threads() < 3:
        pytest.skip("needs >= 3 pool threads")
    assert lib.lsbm_test_pool_helpers(0, 0, 1) == -1
    assert lib.lsbm_test_pool_helpers(16, 3000, 0) == 1  # the caller alone
    assert 1 <= lib.lsbm_test_pool_helpers(16, 3000, 1) <= 2
    assert 1 <= lib.lsbm_test_pool_helpers(16, 3000, 2) <= 3
    assert lib.lsbm_test_pool_helpers(32, 3000, -1) >= 3  # uncapped: the pool joins


_IDLE_PROBE = r"""
import json, sys, time
sys.path.insert(0, sys.argv[1])
from lsbm_amd import _lib
lib = _lib.lib()
if lib.lsbm_host_threads() < 3:
    print(json.dumps({"skip": True}))
    sys.exit(0)
lib.lsbm_test_pool_overlap(1, 2, 2, 1000, None)  # (pool started, workers asleep)
time.sleep(0.05)
c0, w0 = time.process_time(), time.perf_counter()
lib.lsbm_test_pool_overlap(1, 8, 2, 25000, None)  # 8 jobs x 2 pieces of 25 ms
cpu, wall = time.process_time() - c0, time.perf_counter() - w0
c1 = time.process_time()
time.sleep(0.2)
print(json.dumps({"cpu": cpu, "wall": wall, "idle_cpu": time.process_time() - c1}))
"""


def test_pool_idle_workers_do_not_burn_cpu(product_lib):
    """While a job's pieces are all claimed (its caller and one worker each
    running a long piece), the other workers sleep instead of spinning: the
    process's CPU time over 8 such jobs stays a small fraction of one core,
    where round 4's pool kept every worker spinning.
    Measured in a fresh process that loads only the library, so that no
    thread another test left behind (HIP runtime, torch) is counted."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _IDLE_PROBE, repo], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    m = json.loads(r.stdout.strip().splitlines()[-1])
    if m.get("skip"):
        pytest.skip("needs >= 3 pool threads")
    assert m["wall"] >= 0.19, m
    assert m["cpu"] < 0.25 * m["wall"], m
    # and an idle pool costs nothing at all
    assert m["idle_cpu"] < 0.02, m
