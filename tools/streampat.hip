// streampat.hip -- access-pattern probe for the stream-major CRC kernel
// (diagnostic tool, not on the checksum path).
// Build: hipcc --offload-arch=gfx950 -O3 -o build/streampat tools/streampat.hip
//
// Every variant reads a B-byte buffer once per launch as 128-B rows, one 16-B
// non-temporal buffer load per lane per row, 8-lane groups, 1024-thread
// workgroups, one per CU, and spends the CRC row step's work on every row
// (16 conflict-free LDS lookups + the perms/xors).  Only the order in which
// the groups visit the rows differs:
//   fixed   wave w takes 8 consecutive 4 KiB blocks at a time, waves
//           interleaved (the fixed kernel's pattern)
//   window  the buffer is cut into pieces of P bytes, wave w walks pieces
//           w, w + nwaves, ...; inside a piece, rounds of 8 consecutive
//           windows of R rows (group g = window g)
//   segment as window, but inside a piece group g walks the g-th eighth
//           of the piece from start to end, R rows per round
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);        \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

__shared__ uint32_t tab[32768];

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t step(uint32_t c, uint32_t w, uint32_t lb) {
  const uint32_t a0 = __builtin_amdgcn_perm(c, lb, 0x0c020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(c, lb | 0x80u, 0x0c020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(c, lb | 0x10000u, 0x0c020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(c, lb | 0x10080u, 0x0c020700u);
  const char* t = reinterpret_cast<const char*>(tab);
  return xor3(xor3(*(const uint32_t*)(t + a0), *(const uint32_t*)(t + a1), *(const uint32_t*)(t + a2)),
              *(const uint32_t*)(t + a3), w);
}

// mode 0 fixed, 1 window, 2 segment.  P = piece bytes (multiple of 8 R 128).
template <int MODE, int R>
__global__ __launch_bounds__(1024) void k_pat(const uint8_t* __restrict__ base, uint64_t bytes,
                                              uint64_t P, uint32_t* sink) {
  for (int i = threadIdx.x; i < 32768; i += 1024) tab[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, g = lane >> 3, li = lane & 7;
  const uint32_t lb = (lane & 31) << 2;
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * 16;
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  if (MODE == 0) {
    for (uint64_t grp = wave; grp * 32768 < bytes; grp += nw) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint8_t*>(base + grp * 32768), (short)0, 32768, 0x00020000);
      const uint32_t off = g * 4096 + li * 16;
#pragma unroll
      for (int r0 = 0; r0 < 32; r0 += 4) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
          v[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + (r0 + k) * 128, 0, 2));
#pragma unroll
        for (int k = 0; k < 4; k++) {
          c0 = step(c0, v[k].x, lb);
          c1 = step(c1, v[k].y, lb);
          c2 = step(c2, v[k].z, lb);
          c3 = step(c3, v[k].w, lb);
        }
      }
    }
  } else {
    const uint64_t npieces = bytes / P;
    const uint32_t rounds = (uint32_t)(P / (8ull * R * 128));
    for (uint64_t pc = wave; pc < npieces; pc += nw) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint8_t*>(base + pc * P), (short)0, (int)P, 0x00020000);
      for (uint32_t t = 0; t < rounds; t++) {
        const uint32_t off = MODE == 1 ? (t * 8 + g) * (R * 128) + li * 16
                                       : g * (uint32_t)(P / 8) + t * (R * 128) + li * 16;
#pragma unroll
        for (int r0 = 0; r0 < R; r0 += 4) {
          u32x4 v[4];
#pragma unroll
          for (int k = 0; k < 4; k++)
            v[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + (r0 + k) * 128, 0, 2));
#pragma unroll
          for (int k = 0; k < 4; k++) {
            c0 = step(c0, v[k].x, lb);
            c1 = step(c1, v[k].y, lb);
            c2 = step(c2, v[k].z, lb);
            c3 = step(c3, v[k].w, lb);
          }
        }
      }
    }
  }
  if ((c0 ^ c1 ^ c2 ^ c3) == 0x12345678u) sink[0] = c0;
}

template <typename F>
double time_it(F launch, uint64_t bytes) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; i++) launch();
  CK(hipDeviceSynchronize());
  std::vector<float> ms;
  for (int i = 0; i < 7; i++) {
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
  return bytes / (ms[3] * 1e-3) / 1e9;
}

int main(int argc, char** argv) {
  const uint64_t gib = argc > 1 ? strtoull(argv[1], 0, 10) : 16;
  const uint64_t bytes = gib << 30;
  uint8_t* buf;
  uint32_t* sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(buf, 0x5a, bytes));
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("buffer %llu GiB, %d CUs\n", (unsigned long long)gib, cus);
  // spin the clock up
  for (int i = 0; i < 20; i++)
    hipLaunchKernelGGL((k_pat<0, 32>), dim3(cus), dim3(1024), 0, 0, buf, bytes, 0, sink);
  CK(hipDeviceSynchronize());
#define RUN(name, ...) printf("%-40s %8.1f GB/s\n", name, time_it([&] { __VA_ARGS__; }, bytes))
  for (int rep = 0; rep < 2; rep++) {
    RUN("fixed 4KiB x8", hipLaunchKernelGGL((k_pat<0, 32>), dim3(cus), dim3(1024), 0, 0, buf, bytes, 0, sink));
    for (uint64_t P : {32768ull, 131072ull, 1048576ull, 4194304ull}) {
      char nm[64];
      snprintf(nm, 64, "window R16 P=%llu", (unsigned long long)P);
      RUN(nm, hipLaunchKernelGGL((k_pat<1, 16>), dim3(cus), dim3(1024), 0, 0, buf, bytes, P, sink));
      snprintf(nm, 64, "window R32 P=%llu", (unsigned long long)P);
      RUN(nm, hipLaunchKernelGGL((k_pat<1, 32>), dim3(cus), dim3(1024), 0, 0, buf, bytes, P, sink));
      snprintf(nm, 64, "segment R16 P=%llu", (unsigned long long)P);
      RUN(nm, hipLaunchKernelGGL((k_pat<2, 16>), dim3(cus), dim3(1024), 0, 0, buf, bytes, P, sink));
      snprintf(nm, 64, "segment R32 P=%llu", (unsigned long long)P);
      RUN(nm, hipLaunchKernelGGL((k_pat<2, 32>), dim3(cus), dim3(1024), 0, 0, buf, bytes, P, sink));
    }
  }
  // one contiguous piece per wave (bytes / nwaves), as a single-range walk
  const uint64_t nw = (uint64_t)cus * 16;
  const uint64_t Pw = bytes / nw / 32768 * 32768;
  RUN("window R32 P=bytes/nwaves", hipLaunchKernelGGL((k_pat<1, 32>), dim3(cus), dim3(1024), 0, 0, buf, Pw * nw, Pw, sink));
  RUN("segment R32 P=bytes/nwaves", hipLaunchKernelGGL((k_pat<2, 32>), dim3(cus), dim3(1024), 0, 0, buf, Pw * nw, Pw, sink));
  return 0;
}
