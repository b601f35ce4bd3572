// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE / TCC_EA0_RDREQ on
// gfx950 for the access widths of the bloom probe kernels (MI355X_MICROARCH.md
// "HBM": FETCH_SIZE is calibrated only for wide coalesced streams, where it
// reports half the bytes; "other access widths are uncalibrated: calibrate on a
// known byte count in your own access pattern").
//
// Every pattern reads from a 4 GiB buffer (far past the 256 MiB Infinity
// Cache), one launch each, with a known count of distinct 64-B lines touched:
//   stream16   16-B loads per lane, coalesced, over 1 GiB             (guide: x2)
//   gather1    one byte per lane, each at its own random 128-B line  (lines = reads)
//   gather4    one dword per lane, each at its own random 128-B line
//   filter84   per lane one random 84-B "filter" (64-B aligned + 0..20): its
//              first byte and 10 more bytes inside it, as the probe kernel
//              reads them (lines touched counted on the host)
// Prints one JSON line per launch: pattern, reads, distinct 64-B lines and
// 128-B lines touched (computed from the same random positions on the host).
// Run under  rocprofv3 --pmc FETCH_SIZE  (and a pass with
// TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum)  --kernel-trace.
//
//   build: hipcc --offload-arch=gfx950 -O3 -o build/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <set>
#include <vector>

namespace {

constexpr uint64_t kBuf = 4ull << 30;

__host__ __device__ inline uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// i-th random 128-B line of the buffer (distinct with overwhelming probability
// for the counts used here; the host counts the distinct ones exactly)
__host__ __device__ inline uint64_t line_of(uint64_t i, uint64_t seed) { return mix(i ^ seed) % (kBuf / 128); }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ void stream16(const u32x4* __restrict__ p, uint64_t n16, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const u32x4 v = __builtin_nontemporal_load(p + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void gather(const uint8_t* __restrict__ p, uint64_t reads, uint64_t seed, int width,
                       uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < reads; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t a = line_of(i, seed) * 128 + (mix(i) & 63) / width * width;
    acc += width == 1 ? p[a] : *reinterpret_cast<const uint32_t*>(p + (a & ~3ull));
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// the probe kernel's reads of one filter: its last byte (k) and 10 probe bytes
__global__ void filter84(const uint8_t* __restrict__ p, uint64_t filters, uint64_t seed, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < filters; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t f = line_of(i, seed) * 128 + (mix(i) % 21);
    acc += p[f + 83];
    uint32_t h = (uint32_t)mix(i * 7);
    const uint32_t delta = (h >> 17) | (h << 15);
    for (int j = 0; j < 10; j++, h += delta) acc += p[f + (h % 664u) / 8];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

struct Lines {
  size_t l64, l128;
};
Lines count_gather(uint64_t reads, uint64_t seed, int width) {
  std::set<uint64_t> a, b;
  for (uint64_t i = 0; i < reads; i++) {
    const uint64_t x = line_of(i, seed) * 128 + (mix(i) & 63) / width * width;
    a.insert(x / 64);
    b.insert(x / 128);
  }
  return {a.size(), b.size()};
}
Lines count_filter(uint64_t filters, uint64_t seed) {
  std::set<uint64_t> a, b;
  for (uint64_t i = 0; i < filters; i++) {
    const uint64_t f = line_of(i, seed) * 128 + (mix(i) % 21);
    auto add = [&](uint64_t x) {
      a.insert(x / 64);
      b.insert(x / 128);
    };
    add(f + 83);
    uint32_t h = (uint32_t)mix(i * 7);
    const uint32_t delta = (h >> 17) | (h << 15);
    for (int j = 0; j < 10; j++, h += delta) add(f + (h % 664u) / 8);
  }
  return {a.size(), b.size()};
}

}  // namespace

int main() {
  uint8_t* d = nullptr;
  uint32_t* sink = nullptr;
  if (hipMalloc(&d, kBuf) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) {
    fprintf(stderr, "alloc failed\n");
    return 1;
  }
  (void)hipMemset(d, 1, kBuf);
  // flush the Infinity Cache: stream the other 3 GiB first, each pattern's
  // lines are then cold (they are random over 4 GiB)
  const int grid = 256 * 8, block = 256;
  auto flush = [&] {
    hipLaunchKernelGGL(stream16, dim3(grid), dim3(block), 0, 0, reinterpret_cast<const u32x4*>(d + (1ull << 30)),
                       (3ull << 30) / 16, sink);
  };
  flush();
  hipLaunchKernelGGL(stream16, dim3(grid), dim3(block), 0, 0, reinterpret_cast<const u32x4*>(d), (1ull << 30) / 16, sink);
  (void)hipDeviceSynchronize();
  printf("{\"pattern\": \"stream16\", \"bytes\": %llu, \"lines64\": %llu}\n", 1ull << 30, (1ull << 30) / 64);
  const uint64_t reads = 1u << 20;
  for (int width : {1, 4}) {
    flush();
    hipLaunchKernelGGL(gather, dim3(grid), dim3(block), 0, 0, d, reads, (uint64_t)(77 + width), width, sink);
    (void)hipDeviceSynchronize();
    const Lines l = count_gather(reads, 77 + width, width);
    printf("{\"pattern\": \"gather%d\", \"reads\": %llu, \"lines64\": %zu, \"lines128\": %zu}\n", width,
           (unsigned long long)reads, l.l64, l.l128);
  }
  const uint64_t filters = 1u << 19;
  flush();
  hipLaunchKernelGGL(filter84, dim3(grid), dim3(block), 0, 0, d, filters, (uint64_t)99, sink);
  (void)hipDeviceSynchronize();
  const Lines l = count_filter(filters, 99);
  printf("{\"pattern\": \"filter84\", \"filters\": %llu, \"reads\": %llu, \"lines64\": %zu, \"lines128\": %zu}\n",
         (unsigned long long)filters, (unsigned long long)filters * 11, l.l64, l.l128);
  (void)hipFree(d);
  (void)hipFree(sink);
  return 0;
}
