// kbench.cpp — measurement tool (not product): times the C-ABI batch entry
// points on BASELINE configs 2/3/4 with HIP events, without Python/torch in
// the loop, for quick kernel A/B work and rocprofv3 runs.
//
// build: hipcc -O2 --offload-arch=gfx950 -I include tools/kbench.cpp -o tools/kbench -L yustack_amd -lyucsum -ldl -Wl,-rpath,'$ORIGIN/../yustack_amd'
// run:   tools/kbench [config...]   (default 2 3 4; 14 reads KB_LEN)
#include <hip/hip_runtime.h>
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <unistd.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "yucsum.h"
#include <dlfcn.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

__global__ void fill(uint8_t *p, uint64_t n, uint32_t seed) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n / 4; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t x = ((uint32_t)i ^ seed) * 2654435761u;
    x ^= x >> 15;
    x *= 0x2c1b3c6du;
    x ^= x >> 12;
    ((uint32_t *)p)[i] = x;
  }
}

// IPv4 version/IHL byte 0x45 at every packet start (kbench config 12: real headers)
__global__ void set_ihl(uint8_t *p, const uint64_t *off, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (uint64_t)gridDim.x * blockDim.x) p[off[i]] = 0x45;
}

__global__ void set_ihl_stride(uint8_t *p, uint64_t stride, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (uint64_t)gridDim.x * blockDim.x) p[i * stride] = 0x45;
}

// Well-formed TCP/IPv4 datagrams (kbench config 15): IHL 5, TotalLength = the
// packet length, protocol 6, DataOffset 5, as bench config 11 builds them
__global__ void set_dg(uint8_t *p, const uint64_t *off, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t *b = p + off[i];
    const uint64_t len = off[i + 1] - off[i];
    b[0] = 0x45;
    b[2] = (uint8_t)(len >> 8);
    b[3] = (uint8_t)len;
    b[9] = 6;
    if (len > 32) b[32] = 0x50;
  }
}

static void on_segv(int sig) {
  void *bt[64];
  const int k = backtrace(bt, 64);
  fprintf(stderr, "signal %d\n", sig);
  backtrace_symbols_fd(bt, k, 2);
  _exit(128 + sig);
}

int main(int argc, char **argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  signal(SIGSEGV, on_segv);
  std::vector<int> cfgs;
  for (int i = 1; i < argc; ++i) cfgs.push_back(atoi(argv[i]));
  if (cfgs.empty()) cfgs = {2, 3, 4};
  // KB_N: packets per batch (default 1M)
  const uint64_t n = getenv("KB_N") ? strtoull(getenv("KB_N"), nullptr, 10) : 1ull << 20;
  const int reps = 30, rounds = 3;
  // looked up at run time: an A/B against an older library (LD_LIBRARY_PATH=tools/old) lacks it
  typedef const char *(*name_fn)(int, uint64_t);
  const name_fn fill_name = (name_fn)dlsym(RTLD_DEFAULT, "yu_ragged_fill_variant_n");
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint16_t *out, *init;
  uint8_t *addrs;
  CK(hipMalloc(&out, n * 4));  // up to 2 results per packet (YU_MODE_OUTPUTS)
  CK(hipMalloc(&init, n * 2));
  CK(hipMalloc(&addrs, n * 8));
  fill<<<1024, 256>>>((uint8_t *)init, n * 2, 11);
  fill<<<1024, 256>>>(addrs, n * 8, 12);
  for (int cfg : cfgs) {
    uint64_t bytes = 0, alg = 0;
    uint32_t L = 0;
    int mode = 0;
    uint64_t *d_off = nullptr;
    if (cfg == 2) { L = 64; mode = YU_MODE_RAW; bytes = n * L; alg = bytes + 4 * n; }
    if (cfg == 3) { L = 1500; mode = YU_MODE_TCP; bytes = n * L; alg = bytes + 10 * n; }
    // 13: uniform 1M x 1500 B IPv4 datagrams, header checksum only (20-B headers)
    if (cfg == 13) { L = 1500; mode = YU_MODE_IPV4; bytes = n * L; alg = 20 * n + 2 * n; }
    // 14: uniform 1M x KB_LEN-byte UDP datagrams (default 72: 8-B header + 64-B payload)
    if (cfg == 14) {
      L = getenv("KB_LEN") ? (uint32_t)atoi(getenv("KB_LEN")) : 72u;
      mode = YU_MODE_UDP;
      bytes = n * L;
      alg = bytes + 10 * n;
    }
    if ((cfg >= 4 && cfg <= 12) || cfg == 15 || cfg == 16) {
      // 4: BASELINE config 4 (U{64..9000}); 5: tun-like U{64..1500}; 6: U{40..200}
      // (RAW + initial); 7: U{64..1500} TCP segments, 8: U{40..200} UDP (TX kinds, addrs)
      // 9: U{40..600}, 10: U{40..1000} (RAW + initial): small-grid crossover
      const int lo = (cfg == 4 || cfg == 5 || cfg == 7) ? 64 : 40;
      const int hi = cfg == 4 ? 9000 : ((cfg == 5 || cfg == 7 || cfg == 11 || cfg == 12 || cfg == 15) ? 1500 : (cfg == 9 ? 600 : (cfg == 10 ? 1000 : 200)));
      // 11: U{40..1500} IPv4 datagrams, header checksum only (k_rag)
      if (cfg == 11 || cfg == 12) mode = YU_MODE_IPV4;  // 12: IHL 5 in every header
      if (cfg == 7) mode = YU_MODE_TCP;
      if (cfg == 8) mode = YU_MODE_UDP;
      // 15: U{40..1500} well-formed TCP/IPv4 datagrams, both TX fields (bench
      // config 11; KB_MODE=8 verifies the same bytes)
      if (cfg == 15) mode = YU_MODE_TX_DATAGRAM;
      // 16: U{40..200} well-formed datagrams, VERIFY_RX (bench config 7)
      if (cfg == 16) mode = YU_MODE_VERIFY_RX;
      std::mt19937_64 rng(4);
      std::uniform_int_distribution<int> d(lo, hi);
      std::vector<uint64_t> off(n + 1, 0);
      // KB_ALIGN4=1: lengths rounded up to 4 (the in-place writer's contract)
      const bool a4 = getenv("KB_ALIGN4") && atoi(getenv("KB_ALIGN4"));
      for (uint64_t i = 0; i < n; ++i) off[i + 1] = off[i] + (a4 ? (d(rng) + 3) & ~3 : d(rng));
      bytes = off[n];
      alg = bytes + 8 * (n + 1) + (mode == YU_MODE_RAW ? 4 : 10) * n;
      if (cfg == 15) alg = bytes + 8 * (n + 1) + 4 * n;  // two results per datagram
      if (cfg == 16) alg = bytes + 8 * (n + 1) + 2 * n;
      if (mode == YU_MODE_IPV4) alg = 40 * n + 8 * (n + 1) + 2 * n;  // ~mean IHL*4 of random headers
      CK(hipMalloc(&d_off, (n + 1) * 8));
      CK(hipMemcpy(d_off, off.data(), (n + 1) * 8, hipMemcpyHostToDevice));
    }
    // KB_MODE=<0..8> overrides the mode (perf matrix over all modes); addrs for
    // the pseudo-header modes, initial for RAW, nothing for the others
    if (getenv("KB_MODE")) mode = atoi(getenv("KB_MODE"));
    int R = (int)((2ull << 30) / bytes + 1);
    std::vector<uint8_t *> bufs(R);
    for (int r = 0; r < R; ++r) {
      CK(hipMalloc(&bufs[r], bytes + 64));
      fill<<<4096, 256>>>(bufs[r], bytes + 64, 100 + r);
      if (cfg == 12) set_ihl<<<1024, 256>>>(bufs[r], d_off, n);
      if (cfg == 15 || cfg == 16) set_dg<<<1024, 256>>>(bufs[r], d_off, n);
      if (cfg == 13) set_ihl_stride<<<1024, 256>>>(bufs[r], L, n);
    }
    CK(hipDeviceSynchronize());
    // KB_FILL=1: the in-place field writer (TX modes) with no uint16 output
    const bool fill = getenv("KB_FILL") && atoi(getenv("KB_FILL"));
    auto launch = [&](int k) {
      const bool ph = mode == YU_MODE_UDP || mode == YU_MODE_TCP || mode == YU_MODE_VERIFY_TCP ||
                      mode == YU_MODE_VERIFY_UDP;
      const uint16_t *ia = mode == YU_MODE_RAW ? init : nullptr;
      int rc;
      if (fill)
        rc = d_off ? yu_csum_fill_ragged(bufs[k % R], d_off, n, mode, ia, 0, ph ? addrs : nullptr,
                                         nullptr, nullptr)
                   : yu_csum_fill_uniform(bufs[k % R], L, L, n, mode, ia, 0, ph ? addrs : nullptr,
                                          nullptr, nullptr);
      else
        rc = d_off ? yu_csum_batch_ragged(bufs[k % R], d_off, n, mode, ia, 0, ph ? addrs : nullptr,
                                          out, nullptr)
                   : yu_csum_batch_uniform(bufs[k % R], L, L, n, mode, ia, 0, ph ? addrs : nullptr, out,
                                           nullptr);
      if (rc) { fprintf(stderr, "rc %d\n", rc); exit(1); }
    };
    for (int r = 0; r < rounds; ++r) {
      for (int k = 0; k < 3; ++k) launch(k);
      CK(hipEventRecord(e0));
      for (int k = 0; k < reps; ++k) launch(k);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      double s = ms / 1e3 / reps;
      printf("config%d round %d: %8.1f us/launch  %7.1f GB/s alg  (%.3f of 8 TB/s)  %s\n", cfg, r, s * 1e6,
             alg / s / 1e9, alg / s / 8e12,
             d_off ? (fill && fill_name ? fill_name(mode, n) : yu_ragged_variant_n(mode, n))
                   : yu_uniform_variant_n(L, L, n, mode, (uintptr_t)bufs[0] & 15));
    }
    for (auto b : bufs) CK(hipFree(b));
    if (d_off) CK(hipFree(d_off));
  }
  return 0;
}
