// scatter_probe.hip — measurement tool (not product): cost of 1M scattered 2-byte
// stores (one per packet, the checksum field) on their own, after a streaming read
// of the batch, and fused into that read — the in-place writer's memory-side cost.
//
// build: hipcc -O3 --offload-arch=gfx950 tools/scatter_probe.hip -o tools/scatter_probe
// run:   tools/scatter_probe <stride> (default 1500)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

__global__ void scatter(uint8_t *d, uint64_t stride, uint64_t n, uint32_t f, const uint16_t *v) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    *(uint16_t *)(d + i * stride + f) = v[i];
}

__global__ void scatter_nt(uint8_t *d, uint64_t stride, uint64_t n, uint32_t f, const uint16_t *v) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(v[i], (uint16_t *)(d + i * stride + f));
}

// streaming read of the whole batch (dwordx4 per lane), sum kept live
// W-byte aligned block holding each field, written whole by W/16 lanes
template <int W>
__global__ void scatter_block(uint8_t *d, uint64_t stride, uint64_t n, uint32_t f) {
  constexpr int L = W / 16;  // lanes per block
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  for (uint64_t i = t / L; i < n; i += (uint64_t)gridDim.x * blockDim.x / L) {
    uint8_t *b = (uint8_t *)(((uintptr_t)(d + i * stride + f)) & ~(uintptr_t)(W - 1));
    uint4 *q = (uint4 *)b + (t % L);
    *q = make_uint4((uint32_t)i, 1u, 2u, 3u);
  }
}

// W-byte aligned block holding each field, READ, patched with the field's two
// bytes (big-endian v[i]) and written back whole by W/16 lanes: the real bytes of
// a two-pass in-place writer (pass 1 read-only results, pass 2 this)
template <int W, bool NTS>
__global__ void rmw_block(uint8_t *d, uint64_t stride, uint64_t n, uint32_t f, const uint16_t *v) {
  constexpr int L = W / 16;
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  for (uint64_t i = t / L; i < n; i += (uint64_t)gridDim.x * blockDim.x / L) {
    uint8_t *fp = d + i * stride + f;
    uint4 *q = (uint4 *)(((uintptr_t)fp) & ~(uintptr_t)(W - 1)) + (t % L);
    uint4 x = *q;
    const uint64_t off = (uint64_t)(fp - (uint8_t *)q);  // < 16: this lane holds the field
    if (off < 16u) {
      const uint32_t be = (uint32_t)((v[i] >> 8) | ((v[i] & 0xFFu) << 8));
      const uint32_t sh = 8u * (uint32_t)(off & 3u), m = 0xFFFFu << sh;
      const uint32_t k = (uint32_t)(off >> 2);
      uint32_t w = k == 0 ? x.x : (k == 1 ? x.y : (k == 2 ? x.z : x.w));
      w = (w & ~m) | (be << sh);
      if (k == 0) x.x = w; else if (k == 1) x.y = w; else if (k == 2) x.z = w; else x.w = w;
    }
    if (NTS) {
      __builtin_nontemporal_store(x.x, &q->x);
      __builtin_nontemporal_store(x.y, &q->y);
      __builtin_nontemporal_store(x.z, &q->z);
      __builtin_nontemporal_store(x.w, &q->w);
    } else {
      *q = x;
    }
  }
}

typedef unsigned int u4v __attribute__((ext_vector_type(4)));
__global__ void readall(const u4v *d, uint64_t n16, uint32_t *sink) {
  uint32_t s = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const u4v x = __builtin_nontemporal_load(d + i);
    s += x.x ^ x.y ^ x.z ^ x.w;
  }
  if (s == 0x12345678u) sink[0] = s;
}

int main(int argc, char **argv) {
  const uint64_t stride = argc > 1 ? strtoull(argv[1], 0, 10) : 1500;
  const uint64_t n = 1ull << 20, bytes = n * stride;
  uint8_t *d[2];
  uint16_t *v;
  uint32_t *sink;
  for (auto &p : d) CK(hipMalloc(&p, bytes + 64));
  CK(hipMalloc(&v, n * 2));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(v, 0x5a, n * 2));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](const char *what, auto &&f) {
    for (int r = 0; r < 3; ++r) f(r);
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) f(r);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("stride %5lu  %-34s %8.1f us/launch\n", (unsigned long)stride, what, ms * 1e3 / reps);
  };
  const int grid = 256 * 16;
  time("scatter 2-B fields only", [&](int r) { scatter<<<grid, 256>>>(d[r & 1], stride, n, 16, v); });
  time("scatter 2-B fields only, nt", [&](int r) { scatter_nt<<<grid, 256>>>(d[r & 1], stride, n, 16, v); });
  time("stream read only", [&](int r) { readall<<<grid, 256>>>((const u4v *)d[r & 1], bytes / 16, sink); });
  time("stream read, then scatter", [&](int r) {
    readall<<<grid, 256>>>((const u4v *)d[r & 1], bytes / 16, sink);
    scatter<<<grid, 256>>>(d[r & 1], stride, n, 16, v);
  });
  time("stream read, then 32-B blocks", [&](int r) {
    readall<<<grid, 256>>>((const u4v *)d[r & 1], bytes / 16, sink);
    scatter_block<32><<<grid, 256>>>(d[r & 1], stride, n, 16);
  });
  time("stream read, then 64-B blocks", [&](int r) {
    readall<<<grid, 256>>>((const u4v *)d[r & 1], bytes / 16, sink);
    scatter_block<64><<<grid, 256>>>(d[r & 1], stride, n, 16);
  });
  time("stream read, then 128-B lines", [&](int r) {
    readall<<<grid, 256>>>((const u4v *)d[r & 1], bytes / 16, sink);
    scatter_block<128><<<grid, 256>>>(d[r & 1], stride, n, 16);
  });
  time("stream read, then 256-B blocks", [&](int r) {
    readall<<<grid, 256>>>((const u4v *)d[r & 1], bytes / 16, sink);
    scatter_block<256><<<grid, 256>>>(d[r & 1], stride, n, 16);
  });
  time("stream read, then RMW 64-B blocks", [&](int r) {
    readall<<<grid, 256>>>((const u4v *)d[r & 1], bytes / 16, sink);
    rmw_block<64, false><<<grid, 256>>>(d[r & 1], stride, n, 16, v);
  });
  time("stream read, then RMW 64-B blocks, nt", [&](int r) {
    readall<<<grid, 256>>>((const u4v *)d[r & 1], bytes / 16, sink);
    rmw_block<64, true><<<grid, 256>>>(d[r & 1], stride, n, 16, v);
  });
  time("stream read, then RMW 128-B lines", [&](int r) {
    readall<<<grid, 256>>>((const u4v *)d[r & 1], bytes / 16, sink);
    rmw_block<128, false><<<grid, 256>>>(d[r & 1], stride, n, 16, v);
  });
  time("RMW 64-B blocks only", [&](int r) { rmw_block<64, false><<<grid, 256>>>(d[r & 1], stride, n, 16, v); });
  return 0;
}
