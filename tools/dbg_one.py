import ctypes, sys, os
import numpy as np, torch
sys.path.insert(0, os.getcwd())
lib = ctypes.CDLL(sys.argv[1])
torch.cuda.set_device(0)
n = int(sys.argv[2]); L = 128
d = torch.arange(n * L, dtype=torch.int64, device="cuda").to(torch.uint8)
out = torch.full((n,), -1, dtype=torch.int32, device="cuda")
print("init", lib.lsbm_crc32c_init(0))
rc = lib.lsbm_crc32c_fixed_dev(ctypes.c_void_p(d.data_ptr()), ctypes.c_uint64(L), ctypes.c_uint64(L), ctypes.c_uint64(n), None, ctypes.c_void_p(out.data_ptr()), ctypes.c_uint32(0), None)
torch.cuda.synchronize()
print("rc", rc, out.cpu().numpy().view(np.uint32))
