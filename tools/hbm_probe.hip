// hbm_probe.hip — measurement tool (not product): what a plain streaming READ
// reaches on this MI355X, to price the checksum kernel against a known-good
// ceiling instead of only the 8 TB/s datasheet (cdna_hip_programming.md §5.4
// rule 10). Grid-stride dwordx4 loads, U loads in flight per lane, one
// 4-byte store per thread (negligible).
//
// build: hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.hip -o tools/hbm_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void read_sum(const uint4 *__restrict__ p, uint64_t n16, uint32_t *out) {
  uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  uint64_t i = tid;
  for (; i + (U - 1) * nth < n16; i += U * nth) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) {
        u32x4 t = __builtin_nontemporal_load((const u32x4 *)(p + i + u * nth));
        v[u] = make_uint4(t.x, t.y, t.z, t.w);
      } else {
        v[u] = p[i + u * nth];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  for (; i < n16; i += nth) { uint4 v = p[i]; acc += v.x + v.y + v.z + v.w; }
  out[tid] = acc;
}

// Same stream, but every dwordx4 is shifted by `shift` bytes (4-byte aligned,
// not 16-byte aligned) and loaded through a buffer descriptor.
template <int U>
__global__ __launch_bounds__(256) void read_shift(const uint8_t *__restrict__ p, uint64_t n16, uint32_t *out,
                                                  uint32_t shift) {
  uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t i = tid; i + (U - 1) * nth < n16 - 1; i += U * nth) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint8_t *a = p + (i + u * nth) * 16 + shift;
      v[u] = *(const uint4 *)a;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  out[tid] = acc;
}

// k_seg's stream shape: each wave reads 8 KiB tiles (8 dwordx4 per lane), the next
// tile in flight while the current one is summed. LM = false: load u covers the
// tile's u-th KiB (lane L takes 16-byte chunk u*64 + L, k_seg's layout); LM = true:
// lane L takes the 8 consecutive chunks 8L..8L+7 (each load touches 64 lines).
template <bool LM, bool NT>
__global__ __launch_bounds__(256) void read_tile(const uint4 *__restrict__ p, uint64_t n16, uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint64_t ntiles = n16 / 512u;
  uint32_t acc = 0;
  auto ld = [&](uint64_t t, uint4 (&c)[8]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint64_t i = t * 512u + (LM ? lane * 8u + (uint32_t)u : (uint32_t)u * 64u + lane);
      if (NT) {
        const u32x4 v = __builtin_nontemporal_load((const u32x4 *)(p + i));
        c[u] = make_uint4(v.x, v.y, v.z, v.w);
      } else {
        c[u] = p[i];
      }
    }
  };
  uint64_t t = wave;
  if (t < ntiles) {
    uint4 c[8];
    ld(t, c);
    for (; t < ntiles; t += nw) {
      uint4 cn[8];
      ld(t + nw < ntiles ? t + nw : t, cn);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += c[u].x + c[u].y + c[u].z + c[u].w;
#pragma unroll
      for (int u = 0; u < 8; ++u) c[u] = cn[u];
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void fill(uint4 *p, uint64_t n16) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u;
    p[i] = make_uint4(x, x ^ 0x5bd1e995u, x + 7u, ~x);
  }
}

__global__ void copy16(const uint4 *__restrict__ a, uint4 *__restrict__ b, uint64_t n16) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n16; i += (uint64_t)gridDim.x * blockDim.x) b[i] = a[i];
}

typedef void (*RK)(const uint4 *, uint64_t, uint32_t *);

int main(int argc, char **argv) {
  const uint64_t bytes = argc > 1 ? strtoull(argv[1], 0, 10) : 1583349760ull;
  const int reps = 20, rounds = 3;
  // rotating copies: enough that the set exceeds the 256 MiB Infinity Cache
  const int nbuf = argc > 2 ? atoi(argv[2]) : 2;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint64_t n16 = bytes / 16;
  std::vector<uint4 *> buf(nbuf);
  for (int b = 0; b < nbuf; ++b) {
    CK(hipMalloc(&buf[b], n16 * 16));
    fill<<<4096, 256>>>(buf[b], n16);
  }
  uint32_t *out;
  CK(hipMalloc(&out, 64ull << 20));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct K { const char *name; RK fn; } ks[] = {
      {"read U1", read_sum<1, false>}, {"read U2", read_sum<2, false>},
      {"read U4", read_sum<4, false>}, {"read U8", read_sum<8, false>},
      {"read U4 nt", read_sum<4, true>}, {"read U8 nt", read_sum<8, true>},
      {"tile8K u-maj", read_tile<false, false>}, {"tile8K lane-maj", read_tile<true, false>},
      {"tile8K u-maj nt", read_tile<false, true>}, {"tile8K lane-m nt", read_tile<true, true>},
  };
  if (getenv("PROBE_TILES")) {  // only the tile shapes, on k_seg's working grids
    for (int r = 0; r < rounds; ++r)
      for (int i = 6; i < 10; ++i)
        for (int bpc : {3, 4, 8}) {
          int grid = cus * bpc;
          for (int w = 0; w < 3; ++w) ks[i].fn<<<grid, 256>>>(buf[w % nbuf], n16, out);
          CK(hipEventRecord(e0));
          for (int k = 0; k < reps; ++k) ks[i].fn<<<grid, 256>>>(buf[k % nbuf], n16, out);
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          const double sec = ms / 1e3 / reps;
          printf("round %d %-16s blocks/CU %2d: %7.1f us  %7.1f GB/s\n", r, ks[i].name, bpc, sec * 1e6,
                 n16 * 16 / sec / 1e9);
        }
    return 0;
  }
  int bpcs[] = {2, 4, 8, 16};
  printf("buffer %.3f GB x %d rotating, %d CUs\n", bytes / 1e9, nbuf, cus);
  for (int r = 0; r < rounds; ++r) {
    for (auto &k : ks) {
      for (int bpc : bpcs) {
        int grid = cus * bpc;
        for (int w = 0; w < 3; ++w) k.fn<<<grid, 256>>>(buf[w % nbuf], n16, out);
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) k.fn<<<grid, 256>>>(buf[i % nbuf], n16, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        double s = ms / 1e3 / reps;
        printf("round %d %-12s blocks/CU %2d: %7.1f us  %7.1f GB/s\n", r, k.name, bpc, s * 1e6,
               n16 * 16 / s / 1e9);
      }
    }
    for (uint32_t shift : {0u, 4u, 8u}) {
      for (int bpc : {4, 8}) {
        int grid = cus * bpc;
        for (int w = 0; w < 3; ++w) read_shift<2><<<grid, 256>>>((const uint8_t *)buf[w % nbuf], n16, out, shift);
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) read_shift<2><<<grid, 256>>>((const uint8_t *)buf[i % nbuf], n16, out, shift);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        double s = ms / 1e3 / reps;
        printf("round %d read U2 shift %u blocks/CU %d: %7.1f us  %7.1f GB/s\n", r, shift, bpc, s * 1e6,
               n16 * 16 / s / 1e9);
      }
    }
    {  // copy: read+write
      uint64_t h = n16 / 2;
      for (int w = 0; w < 3; ++w) copy16<<<cus * 8, 256>>>(buf[0], buf[1], h);
      CK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) copy16<<<cus * 8, 256>>>(buf[i % 2], buf[(i + 1) % 2], h);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      double s = ms / 1e3 / reps;
      printf("round %d copy16 (r+w)        : %7.1f us  %7.1f GB/s\n", r, s * 1e6, 2.0 * h * 16 / s / 1e9);
    }
  }
  return 0;
}
