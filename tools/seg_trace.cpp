// seg_trace.cpp — measurement tool (not product): per-step timeline of k_seg on a
// small-packet ragged batch (kbench config 16: 1M U{40..200} VERIFY_RX datagrams),
// from s_memtime stamps the DEBUG side build records for every 61st wave: step start,
// after the next chunk's geometry/offset loads, after the next tile's loads are issued
// (and the current tile's first chunk has landed), after its last chunk has landed,
// end of step. Side build: tools/side_build.sh tools/old HEAD tools/seg_trace_patch.py
// build: hipcc -O2 --offload-arch=gfx950 -I include tools/seg_trace.cpp -o tools/seg_trace -L tools/old -lyucsum -Wl,-rpath,'$ORIGIN/old'
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <random>
#include <vector>

#include "yucsum.h"

extern "C" void yu_debug_set_trace(uint64_t *p);

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

__global__ void fill(uint8_t *p, uint64_t n, uint32_t seed) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n / 4; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t x = ((uint32_t)i ^ seed) * 2654435761u;
    x ^= x >> 15; x *= 0x2c1b3c6du; x ^= x >> 12;
    ((uint32_t *)p)[i] = x;
  }
}
__global__ void set_dg(uint8_t *p, const uint64_t *off, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t *b = p + off[i];
    const uint64_t len = off[i + 1] - off[i];
    b[0] = 0x45; b[2] = (uint8_t)(len >> 8); b[3] = (uint8_t)len; b[9] = 6;
  }
}

int main(int argc, char **argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : (1ull << 20);
  const int hi = argc > 2 ? atoi(argv[2]) : 200;
  const int mode = argc > 3 ? atoi(argv[3]) : YU_MODE_VERIFY_RX;
  std::mt19937_64 rng(4);
  std::uniform_int_distribution<int> d(40, hi);
  std::vector<uint64_t> off(n + 1, 0);
  for (uint64_t i = 0; i < n; ++i) off[i + 1] = off[i] + d(rng);
  const uint64_t bytes = off[n];
  const int R = (int)((2ull << 30) / bytes + 1);
  uint64_t *d_off; uint16_t *out;
  CK(hipMalloc(&d_off, (n + 1) * 8));
  CK(hipMemcpy(d_off, off.data(), (n + 1) * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&out, n * 4));
  std::vector<uint8_t *> bufs(R);
  for (auto &b : bufs) { CK(hipMalloc(&b, bytes + 64)); fill<<<4096, 256>>>(b, bytes + 64, 7); set_dg<<<1024, 256>>>(b, d_off, n); }
  const uint64_t nsamp = 65536 / 61 + 2, ntr = nsamp * 64 * 8;
  uint64_t *tr;
  CK(hipMalloc(&tr, ntr * 8));
  CK(hipMemset(tr, 0, ntr * 8));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int k = 0; k < 20; ++k) yu_csum_batch_ragged(bufs[k % R], d_off, n, mode, nullptr, 0, nullptr, out, nullptr);
  yu_debug_set_trace(tr);
  CK(hipEventRecord(e0));
  int rc = yu_csum_batch_ragged(bufs[20 % R], d_off, n, mode, nullptr, 0, nullptr, out, nullptr);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  yu_debug_set_trace(nullptr);
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<uint64_t> h(ntr);
  CK(hipMemcpy(h.data(), tr, ntr * 8, hipMemcpyDeviceToHost));
  printf("n %lu  U{40..%d}  mode %d  rc %d  traced launch %.1f us  kernel %s\n", (unsigned long)n, hi, mode, rc,
         ms * 1e3, yu_ragged_variant_n(mode, n));
  // segments between the 7 stamps of a step (ticks = shader clock cycles)
  // kind 0/1 (scan path: mid / last step): ... scans, park/points, epilogue;
  // kind 2 (one-tile chunk summed per lane): ... park, range sums, parse + results
  const char *seg[6] = {"geom+offs", "tile issue+wait c0", "wait rest", "scans|park", "points|sums", "epilogue|parse"};
  struct Acc { double s[6] = {0, 0, 0, 0, 0, 0}; double tot = 0; int cnt = 0; };
  Acc last_a, mid_a, ls_a;
  double gaps[2] = {0, 0}; int ngaps[2] = {0, 0};
  std::vector<double> starts, ends;
  for (uint64_t w = 0; w < nsamp; ++w) {
    for (int k = 0; k < 64; ++k) {
      const uint64_t *q = &h[(w * 64 + k) * 8];
      if (!q[0]) break;
      Acc &a = (q[7] & 0xFF) == 2 ? ls_a : ((q[7] & 0xFF) ? last_a : mid_a);
      for (int j = 0; j < 6; ++j) a.s[j] += (double)(int64_t)(q[j + 1] - q[j]);
      a.tot += (double)(int64_t)(q[6] - q[0]);
      a.cnt++;
      if (k > 0) {  // gap from the previous step's last stamp to this step's first
        const uint64_t *pq = &h[(w * 64 + k - 1) * 8];
        gaps[(pq[7] & 0xFF) ? 1 : 0] += (double)(int64_t)(q[0] - pq[6]);
        ngaps[(pq[7] & 0xFF) ? 1 : 0]++;
      }
      if (k == 0) starts.push_back((double)q[0]);
      if (k == 63 || !h[(w * 64 + k + 1) * 8]) ends.push_back((double)q[6]);
    }
  }
  auto pr = [&](const char *name, const Acc &a) {
    if (!a.cnt) return;
    printf("%-11s n=%5d", name, a.cnt);
    for (int j = 0; j < 6; ++j) printf("  %s %6.0f", seg[j], a.s[j] / a.cnt);
    printf("  | step %6.0f\n", a.tot / a.cnt);
  };
  pr("last steps", last_a);
  pr("mid steps", mid_a);
  pr("lane chunks", ls_a);
  printf("gap to the next step's start: after a mid step %.0f ticks (n=%d), after a chunk's last step %.0f (n=%d)\n",
         ngaps[0] ? gaps[0] / ngaps[0] : 0.0, ngaps[0], ngaps[1] ? gaps[1] / ngaps[1] : 0.0, ngaps[1]);
  std::sort(starts.begin(), starts.end());
  std::sort(ends.begin(), ends.end());
  if (!starts.empty()) {
    const double t0 = starts[starts.size() / 20];
    printf("wave first-step start (ticks after the 5th-percentile start): p50 %.0f p95 %.0f; last-step end: p5 %.0f p50 %.0f p95 %.0f max %.0f\n",
           starts[starts.size() / 2] - t0, starts[starts.size() * 95 / 100] - t0, ends[ends.size() / 20] - t0,
           ends[ends.size() / 2] - t0, ends[ends.size() * 95 / 100] - t0, ends.back() - t0);
  }
  return 0;
}
