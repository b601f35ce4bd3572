// membench.hip -- read-bandwidth ceiling probes on gfx950 (diagnostic tool).
// Build: hipcc --offload-arch=gfx950 -O3 -o build/membench tools/membench.hip
// Each variant streams a B-byte device buffer once per launch; reports GB/s
// (median of 10 launches after 3 warmups, hipEvent timing).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

// 1. grid-stride, U loads in flight per thread, optional nt
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_stream(const u32x4* __restrict__ p, uint64_t n16,
                                                uint32_t* sink) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  uint64_t i = tid;
  for (; i + (U - 1) * nt < n16; i += U * nt) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; k++) v[k] = NT ? __builtin_nontemporal_load(p + i + k * nt) : p[i + k * nt];
#pragma unroll
    for (int k = 0; k < U; k++) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  for (; i < n16; i += nt) acc ^= p[i].x;
  if (acc == 0x12345678u) sink[0] = acc;
}

// 2. the CRC kernel's access pattern: 1024-thread WGs, 8-lane groups read
//    128-B rows of 8 different 4 KiB blocks; persistent over block groups.
template <int PF, bool NT>
__global__ __launch_bounds__(1024) void k_rows(const uint8_t* __restrict__ base, uint64_t nblocks,
                                               uint32_t* sink) {
  const uint32_t lane = threadIdx.x & 63, g = lane >> 3, li = lane & 7;
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * 16;
  uint32_t acc = 0;
  for (uint64_t grp = wave; grp * 8 < nblocks; grp += nw) {
    const u32x4* p = reinterpret_cast<const u32x4*>(base + (grp * 8 + g) * 4096) + li;
#pragma unroll
    for (int r0 = 0; r0 < 32; r0 += PF) {
      u32x4 v[PF];
#pragma unroll
      for (int k = 0; k < PF; k++) v[k] = NT ? __builtin_nontemporal_load(p + (r0 + k) * 8) : p[(r0 + k) * 8];
#pragma unroll
      for (int k = 0; k < PF; k++) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// 2b. rows pattern + synthetic per-row work: WORK dependent-ish VALU ops per
//     row and LDS lookups (16 conflict-free ds_read_b32 per row), buffer or global loads.
template <int PF, bool BUF, int VALU, bool LDS>
__global__ __launch_bounds__(1024) void k_rows_work(const uint8_t* __restrict__ base,
                                                    uint64_t nblocks, uint32_t* sink) {
  __shared__ uint32_t tab[32768];
  for (int i = threadIdx.x; i < 32768; i += 1024) tab[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, g = lane >> 3, li = lane & 7;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + wv;
  const uint64_t nw = (uint64_t)gridDim.x * 16;
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  const uint32_t lb = (lane & 31) << 2;
  for (uint64_t grp = wave; grp * 8 < nblocks; grp += nw) {
    const uint8_t* wb = base + grp * 8 * 4096;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(wb), (short)0, 0x7fffffff, 0x00020000);
    const uint32_t loff = g * 4096 + li * 16;
#pragma unroll
    for (int r0 = 0; r0 < 32; r0 += PF) {
      u32x4 v[PF];
#pragma unroll
      for (int k = 0; k < PF; k++)
        v[k] = BUF ? __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, loff + (r0 + k) * 128, 0, 2))
                   : __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wb + loff + (r0 + k) * 128));
#pragma unroll
      for (int k = 0; k < PF; k++) {
        c0 ^= v[k].x; c1 ^= v[k].y; c2 ^= v[k].z; c3 ^= v[k].w;
#pragma unroll
        for (int j = 0; j < VALU / 4; j++) {
          c0 = __builtin_amdgcn_perm(c0, lb, 0x0c020400u + j);
          c1 = __builtin_amdgcn_perm(c1, lb, 0x0c020500u + j);
          c2 = __builtin_amdgcn_perm(c2, lb, 0x0c020600u + j);
          c3 = __builtin_amdgcn_perm(c3, lb, 0x0c020700u + j);
        }
        if (LDS) {
          uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
#pragma unroll
          for (int q = 0; q < 4; q++) {
            t0 ^= tab[((c0 >> (8 * q)) & 0xff) * 32 + (lane & 31) + q * 8192];
            t1 ^= tab[((c1 >> (8 * q)) & 0xff) * 32 + (lane & 31) + q * 8192];
            t2 ^= tab[((c2 >> (8 * q)) & 0xff) * 32 + (lane & 31) + q * 8192];
            t3 ^= tab[((c3 >> (8 * q)) & 0xff) * 32 + (lane & 31) + q * 8192];
          }
          c0 = t0; c1 = t1; c2 = t2; c3 = t3;
        }
      }
    }
  }
  if ((c0 ^ c1 ^ c2 ^ c3) == 0x12345678u) sink[0] = c0;
}

// 2c. narrower groups: LPB lanes per 4 KiB block, each lane 16 B per row of
//     LPB*16 bytes; 64/LPB blocks per wave-instruction.
template <int LPB, int PF>
__global__ __launch_bounds__(1024) void k_rows_lpb(const uint8_t* __restrict__ base,
                                                   uint64_t nblocks, uint32_t* sink) {
  constexpr int BPW = 64 / LPB, ROWB = LPB * 16, NROW = 4096 / ROWB;
  const uint32_t lane = threadIdx.x & 63, g = lane / LPB, li = lane % LPB;
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * 16;
  uint32_t acc = 0;
  for (uint64_t grp = wave; grp * BPW < nblocks; grp += nw) {
    const u32x4* p = reinterpret_cast<const u32x4*>(base + (grp * BPW + g) * 4096 + li * 16);
#pragma unroll
    for (int r0 = 0; r0 < NROW; r0 += PF) {
      u32x4 v[PF];
#pragma unroll
      for (int k = 0; k < PF; k++) v[k] = __builtin_nontemporal_load(p + (r0 + k) * (ROWB / 16));
#pragma unroll
      for (int k = 0; k < PF; k++) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// 3. LDS-DMA: each wave streams 1 KiB pieces into a DEPTH-slot LDS ring with
//    global_load_lds_dwordx4, then reads each slot back (ds_read_b128).
#define STR2(x) #x
#define STR(x) STR2(x)
template <int DEPTH, int AUX>
__global__ __launch_bounds__(1024) void k_ldsdma(const u32x4* __restrict__ p, uint64_t n1k,
                                                 uint32_t* sink) {
  extern __shared__ __attribute__((aligned(16))) u32x4 ring[];  // 16 waves * DEPTH * 64
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  u32x4* my = ring + w * DEPTH * 64;
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + w;
  const uint64_t nw = (uint64_t)gridDim.x * 16;
  uint32_t acc = 0;
  // piece j of this wave = global piece wave + j*nw
  uint64_t niter = n1k > wave ? (n1k - wave + nw - 1) / nw : 0;
  for (uint64_t j = 0; j < niter + DEPTH - 1; j++) {
    if (j < niter) {
      const u32x4* src = p + (wave + j * nw) * 64 + lane;
      __builtin_amdgcn_global_load_lds(src, my + (j % DEPTH) * 64, 16, 0, AUX);
    }
    if (j >= DEPTH - 1) {
      if (j < niter) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH - 1) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      const u32x4 v = my[((j - (DEPTH - 1)) % DEPTH) * 64 + lane];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// 4. raw buffer loads with cache-policy aux bits
template <int U, int AUX>
__global__ __launch_bounds__(256) void k_buffer(const uint8_t* __restrict__ p, uint64_t n16,
                                                uint32_t* sink) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  // one descriptor per 2 GiB window
  for (uint64_t win = 0; win * (1ull << 27) < n16; win++) {
    const uint64_t w0 = win << 27, w1 = std::min<uint64_t>(n16, (win + 1) << 27);
    __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p + w0 * 16), (short)0, (int)((w1 - w0) * 16 > 0x7fffffffull ? 0x7fffffff : (w1 - w0) * 16), 0x00020000);
    uint64_t i = tid;
    for (; w0 + i + (U - 1) * nt < w1; i += U * nt) {
      u32x4 v[U];
#pragma unroll
      for (int k = 0; k < U; k++)
        v[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)((i + k * nt) * 16), 0, AUX));
#pragma unroll
      for (int k = 0; k < U; k++) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <typename F>
double time_it(F launch, uint64_t bytes) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; i++) launch();
  CK(hipDeviceSynchronize());
  std::vector<float> ms;
  for (int i = 0; i < 10; i++) {
    CK(hipEventRecord(a, 0));
    launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float t;
    CK(hipEventElapsedTime(&t, a, b));
    ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  CK(hipGetLastError());
  return bytes / (ms[5] * 1e-3) / 1e9;
}

int main(int argc, char** argv) {
  const uint64_t gib = argc > 1 ? strtoull(argv[1], 0, 10) : 4;
  const uint64_t bytes = gib << 30;
  uint8_t* buf;
  uint32_t* sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(buf, 0x5a, bytes));
  const u32x4* p = reinterpret_cast<const u32x4*>(buf);
  const uint64_t n16 = bytes / 16;
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("buffer %llu GiB, %d CUs\n", (unsigned long long)gib, cus);
#define RUN(name, ...) printf("%-36s %8.1f GB/s\n", name, time_it([&] { __VA_ARGS__; }, bytes))
  for (int wgs_per_cu : {4, 8, 16}) {
    const int grid = cus * wgs_per_cu;
    char nm[64];
    snprintf(nm, 64, "stream U4 nt   grid=%dx", wgs_per_cu);
    RUN(nm, hipLaunchKernelGGL((k_stream<4, true>), dim3(grid), dim3(256), 0, 0, p, n16, sink));
    snprintf(nm, 64, "stream U8 nt   grid=%dx", wgs_per_cu);
    RUN(nm, hipLaunchKernelGGL((k_stream<8, true>), dim3(grid), dim3(256), 0, 0, p, n16, sink));
    snprintf(nm, 64, "stream U8 plain grid=%dx", wgs_per_cu);
    RUN(nm, hipLaunchKernelGGL((k_stream<8, false>), dim3(grid), dim3(256), 0, 0, p, n16, sink));
    snprintf(nm, 64, "buffer U8 aux0 grid=%dx", wgs_per_cu);
    RUN(nm, hipLaunchKernelGGL((k_buffer<8, 0>), dim3(grid), dim3(256), 0, 0, buf, n16, sink));
    snprintf(nm, 64, "buffer U8 aux2 grid=%dx", wgs_per_cu);
    RUN(nm, hipLaunchKernelGGL((k_buffer<8, 2>), dim3(grid), dim3(256), 0, 0, buf, n16, sink));
  }
  const uint64_t nblocks = bytes / 4096;
  for (int g : {1, 2}) {
    char nm[64];
    snprintf(nm, 64, "rows PF8 nt   wg/cu=%d", g);
    RUN(nm, hipLaunchKernelGGL((k_rows<8, true>), dim3(cus * g), dim3(1024), 0, 0, buf, nblocks, sink));
    snprintf(nm, 64, "rows PF8 plain wg/cu=%d", g);
    RUN(nm, hipLaunchKernelGGL((k_rows<8, false>), dim3(cus * g), dim3(1024), 0, 0, buf, nblocks, sink));
    snprintf(nm, 64, "rows PF16 nt  wg/cu=%d", g);
    RUN(nm, hipLaunchKernelGGL((k_rows<16, true>), dim3(cus * g), dim3(1024), 0, 0, buf, nblocks, sink));
    snprintf(nm, 64, "rows PF4 nt   wg/cu=%d", g);
    RUN(nm, hipLaunchKernelGGL((k_rows<4, true>), dim3(cus * g), dim3(1024), 0, 0, buf, nblocks, sink));
  }
  {
    char nm[64];
#define RW(PF, BUF, VALU, LDS)                                                           \
    snprintf(nm, 64, "rowswork pf%d buf%d valu%d lds%d", PF, BUF, VALU, LDS);           \
    RUN(nm, hipLaunchKernelGGL((k_rows_work<PF, BUF, VALU, LDS>), dim3(cus), dim3(1024), 0, 0, buf, \
                               nblocks, sink));
    RW(4, 0, 0, 0)
    RW(4, 1, 0, 0)
    RW(4, 0, 16, 0)
    RW(4, 1, 16, 0)
    RW(4, 0, 32, 0)
    RW(4, 0, 0, 1)
    RW(4, 1, 0, 1)
    RW(4, 0, 16, 1)
    RW(4, 1, 16, 1)
    RW(8, 1, 16, 1)
    RW(2, 1, 16, 1)
  }
  RUN("rows lpb8 pf4", hipLaunchKernelGGL((k_rows_lpb<8, 4>), dim3(cus), dim3(1024), 0, 0, buf, nblocks, sink));
  RUN("rows lpb4 pf4", hipLaunchKernelGGL((k_rows_lpb<4, 4>), dim3(cus), dim3(1024), 0, 0, buf, nblocks, sink));
  RUN("rows lpb4 pf8", hipLaunchKernelGGL((k_rows_lpb<4, 8>), dim3(cus), dim3(1024), 0, 0, buf, nblocks, sink));
  RUN("rows lpb2 pf8", hipLaunchKernelGGL((k_rows_lpb<2, 8>), dim3(cus), dim3(1024), 0, 0, buf, nblocks, sink));
  RUN("rows lpb16 pf4", hipLaunchKernelGGL((k_rows_lpb<16, 4>), dim3(cus), dim3(1024), 0, 0, buf, nblocks, sink));
  RUN("rows lpb64 pf4", hipLaunchKernelGGL((k_rows_lpb<64, 4>), dim3(cus), dim3(1024), 0, 0, buf, nblocks, sink));
  const uint64_t n1k = bytes / 1024;
#define DMA(D, AUX)                                                                              \
  do {                                                                                           \
    char nm[64];                                                                                 \
    snprintf(nm, 64, "ldsdma depth=%d aux=%d", D, AUX);                                          \
    RUN(nm, hipLaunchKernelGGL((k_ldsdma<D, AUX>), dim3(cus), dim3(1024), 16 * D * 1024, 0, p, \
                               n1k, sink));                                                      \
  } while (0)
  CK(hipFuncSetAttribute((const void*)k_ldsdma<8, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void*)k_ldsdma<8, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void*)k_ldsdma<4, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void*)k_ldsdma<2, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  DMA(2, 2);
  DMA(4, 2);
  DMA(8, 0);
  DMA(8, 2);
  return 0;
}
