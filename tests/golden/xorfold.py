"""XOR of all rows of a 2-D integer tensor, folded on the device.

Test infrastructure for the full-size linearity checks
(tests/test_gpu_parity.py::crc_linearity_holds, bench.py --dump-samples):
for blocks of one length, crc32c::Value is an affine map over GF(2), so the
XOR of a batch's CRCs is pinned by the oracle's CRC of the XOR of its blocks.
"""


def xor_fold_rows(x):
    import torch
    acc = torch.zeros(x.shape[1], dtype=x.dtype, device=x.device)
    while x.shape[0] > 1:
        h = x.shape[0] // 2
        if x.shape[0] % 2:
            acc ^= x[-1]
        x = x[:h] ^ x[h:2 * h]
    return acc ^ x[0] if x.shape[0] else acc
