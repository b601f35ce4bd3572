"""Run the ragged path of one geometry against a chosen library build and the oracle."""
import ctypes, sys, os
import numpy as np, torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from conftest import Oracle
from golden.splitmix import stream_bytes
lib = ctypes.CDLL(sys.argv[1])
L, stride, n = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
torch.cuda.set_device(0)
data = stream_bytes(777 + L, 0, (n - 1) * stride + L)
d = torch.from_numpy(data).to("cuda")
out = torch.full((n,), -1, dtype=torch.int32, device="cuda")
print("init", lib.lsbm_crc32c_init(0), flush=True)
rc = lib.lsbm_crc32c_fixed_dev(ctypes.c_void_p(d.data_ptr()), ctypes.c_uint64(stride), ctypes.c_uint64(L), ctypes.c_uint64(n), None, ctypes.c_void_p(out.data_ptr()), ctypes.c_uint32(0), None)
torch.cuda.synchronize()
got = out.cpu().numpy().view(np.uint32)
o = Oracle(os.path.join(os.getcwd(), "oracle", "liboracle_crc32c.so"))
want = o.batch_fixed(data, stride, L, n)
print("rc", rc, "mismatches", int((got != want).sum()), "of", n, flush=True)
