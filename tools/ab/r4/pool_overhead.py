"""Worker-pool overhead per parallel_for on this machine (no GPU needed):
lsbm_test_pool_overlap(1 caller, N jobs, P empty pieces) -> us per job."""
import ctypes, os, sys
L = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "..", "..", "..", "lsbm_amd", "liblsbm_crc32c.so"))
L.lsbm_test_pool_overlap.argtypes = [ctypes.c_int] * 4 + [ctypes.POINTER(ctypes.c_double)]
print("threads", L.lsbm_host_threads())
for rep in range(2):
    for pieces in (2, 8, 16, 32, 64):
        s = ctypes.c_double()
        L.lsbm_test_pool_overlap(1, 5000, pieces, 0, ctypes.byref(s))
        print(rep, pieces, "pieces: %.2f us per job" % (s.value / 5000 * 1e6), flush=True)
