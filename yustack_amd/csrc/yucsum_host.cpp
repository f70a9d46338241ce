// yucsum_host.cpp — host-memory batched entry point (yu_csum_batch_host_uniform).
//
// yustack's packets start and end in host memory: the tun link endpoint
// reads into Go slices (link/tundev/tundev.go:78-151) and writes them back
// with writev (:171-196). This path moves a host batch through the GPU:
//
//   slice k:  [CPU memcpy -> pinned staging]  (skipped when the caller's
//             buffer is already pinned)
//             H2D hipMemcpyAsync -> checksum kernel -> D2H hipMemcpyAsync
//
// on one of three staging slots, each with its own stream, so the H2D of
// slice k+1, the kernel of slice k and the D2H of slice k-1 overlap, and
// the CPU staging copy of the next slice overlaps all of them. Staging
// buffers are per (calling thread, device) and grow on demand; nothing is
// shared between threads, so concurrent callers need no lock.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <string.h>

#include <memory>

#include "yucsum.h"

namespace {

constexpr int kSlots = 3;
constexpr uint64_t kSliceBytes = 32ull << 20;

int hip_rc(hipError_t e) {
  if (e == hipSuccess) return YU_OK;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return YU_ENODEV;
  if (e == hipErrorOutOfMemory) return YU_ENOMEM;
  return YU_EHIP_BASE - (int)e;
}

#define YU_TRY(expr)                  \
  do {                                \
    hipError_t _e = (expr);           \
    if (_e != hipSuccess) return hip_rc(_e); \
  } while (0)

struct Slot {
  uint8_t *h_data = nullptr, *h_addrs = nullptr;
  uint16_t *h_init = nullptr, *h_out = nullptr;
  uint8_t *d_data = nullptr, *d_addrs = nullptr;
  uint16_t *d_init = nullptr, *d_out = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t done = nullptr;
  uint64_t first = 0, cnt = 0;
  bool busy = false, staged_out = false;
};

struct Ctx {
  int dev = -1;
  uint64_t cap_data = 0, cap_pk = 0;
  Slot s[kSlots];

  void release() {
    for (Slot &x : s) {
      if (x.h_data) (void)hipHostFree(x.h_data);
      if (x.h_addrs) (void)hipHostFree(x.h_addrs);
      if (x.h_init) (void)hipHostFree(x.h_init);
      if (x.h_out) (void)hipHostFree(x.h_out);
      if (x.d_data) (void)hipFree(x.d_data);
      if (x.d_addrs) (void)hipFree(x.d_addrs);
      if (x.d_init) (void)hipFree(x.d_init);
      if (x.d_out) (void)hipFree(x.d_out);
      if (x.done) (void)hipEventDestroy(x.done);
      if (x.st) (void)hipStreamDestroy(x.st);
      x = Slot();
    }
    cap_data = cap_pk = 0;
  }
  ~Ctx() {
    if (dev >= 0 && hipSetDevice(dev) == hipSuccess) release();
  }

  int reserve(uint64_t data_bytes, uint64_t pk) {
    if (data_bytes <= cap_data && pk <= cap_pk) return YU_OK;
    release();
    for (Slot &x : s) {
      YU_TRY(hipStreamCreateWithFlags(&x.st, hipStreamNonBlocking));
      YU_TRY(hipEventCreateWithFlags(&x.done, hipEventDisableTiming));
      YU_TRY(hipHostMalloc((void **)&x.h_data, data_bytes ? data_bytes : 16, 0));
      YU_TRY(hipHostMalloc((void **)&x.h_addrs, pk * 8, 0));
      YU_TRY(hipHostMalloc((void **)&x.h_init, pk * 2, 0));
      YU_TRY(hipHostMalloc((void **)&x.h_out, pk * 2, 0));
      YU_TRY(hipMalloc((void **)&x.d_data, data_bytes ? data_bytes : 16));
      YU_TRY(hipMalloc((void **)&x.d_addrs, pk * 8));
      YU_TRY(hipMalloc((void **)&x.d_init, pk * 2));
      YU_TRY(hipMalloc((void **)&x.d_out, pk * 2));
    }
    cap_data = data_bytes;
    cap_pk = pk;
    return YU_OK;
  }
};

thread_local std::unique_ptr<Ctx> t_ctx[64];

bool is_pinned(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky "invalid value" for pageable
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

int finish(Slot &x, uint16_t *h_out) {
  if (!x.busy) return YU_OK;
  YU_TRY(hipEventSynchronize(x.done));
  if (x.staged_out) memcpy(h_out + x.first, x.h_out, x.cnt * 2);
  x.busy = false;
  return YU_OK;
}

int run(const uint8_t *h_data, uint64_t stride, uint32_t len, uint64_t n,
        int mode, const uint16_t *h_init, uint16_t initial,
        const uint8_t *h_addrs, uint16_t *h_out, int device) {
  std::unique_ptr<Ctx> &cp = t_ctx[device];
  if (!cp) {
    cp.reset(new Ctx());
    cp->dev = device;
  }
  Ctx &c = *cp;
  // A previous call that failed midway may have left slices in flight:
  // drain them without copying (their h_out belonged to that call).
  for (Slot &x : c.s) {
    if (x.busy) (void)hipEventSynchronize(x.done);
    x.busy = false;
  }
  const uint64_t pstride = stride ? stride : 1;
  uint64_t slice = kSliceBytes / pstride;
  if (slice < 1) slice = 1;
  if (slice > n) slice = n;
  const uint64_t data_bytes = (slice - 1) * stride + len;
  int rc = c.reserve(data_bytes, slice);
  if (rc) return rc;

  const bool pin_in = is_pinned(h_data);
  const bool pin_out = is_pinned(h_out);
  uint64_t k = 0;
  for (uint64_t first = 0; first < n; first += slice, ++k) {
    Slot &x = c.s[k % kSlots];
    rc = finish(x, h_out);
    if (rc) return rc;
    const uint64_t cnt = (n - first) < slice ? (n - first) : slice;
    const uint64_t bytes = (cnt - 1) * stride + len;
    const uint8_t *src = h_data + first * stride;
    if (!pin_in && bytes) {
      memcpy(x.h_data, src, bytes);
      src = x.h_data;
    }
    if (bytes) YU_TRY(hipMemcpyAsync(x.d_data, src, bytes, hipMemcpyHostToDevice, x.st));
    const uint16_t *d_init = nullptr;
    const uint8_t *d_addrs = nullptr;
    if (h_init) {
      memcpy(x.h_init, h_init + first, cnt * 2);
      YU_TRY(hipMemcpyAsync(x.d_init, x.h_init, cnt * 2, hipMemcpyHostToDevice, x.st));
      d_init = x.d_init;
    }
    if (h_addrs) {
      memcpy(x.h_addrs, h_addrs + first * 8, cnt * 8);
      YU_TRY(hipMemcpyAsync(x.d_addrs, x.h_addrs, cnt * 8, hipMemcpyHostToDevice, x.st));
      d_addrs = x.d_addrs;
    }
    rc = yu_csum_batch_uniform(x.d_data, stride, len, cnt, mode, d_init,
                               initial, d_addrs, x.d_out, x.st);
    if (rc) return rc;
    x.staged_out = !pin_out;
    YU_TRY(hipMemcpyAsync(pin_out ? h_out + first : x.h_out, x.d_out, cnt * 2,
                          hipMemcpyDeviceToHost, x.st));
    YU_TRY(hipEventRecord(x.done, x.st));
    x.first = first;
    x.cnt = cnt;
    x.busy = true;
  }
  for (Slot &x : c.s) {
    rc = finish(x, h_out);
    if (rc) return rc;
  }
  return YU_OK;
}

}  // namespace

extern "C" int yu_csum_batch_host_uniform(const uint8_t *h_data,
                                          uint64_t stride, uint32_t len,
                                          uint64_t n, int mode,
                                          const uint16_t *h_initial_arr,
                                          uint16_t initial,
                                          const uint8_t *h_addrs,
                                          uint16_t *h_out, int device) {
  if (mode < 0 || mode >= YU_MODE_COUNT || !h_out) return YU_EINVAL;
  if (n == 0) return YU_OK;
  if (!h_data && len) return YU_EINVAL;
  if (mode != YU_MODE_RAW && len > YU_MAX_TRANSPORT_LEN) return YU_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return YU_ENODEV;
  if (device < 0 || device >= ndev || device >= 64) return YU_ENODEV;
  int prev = 0;
  YU_TRY(hipGetDevice(&prev));
  YU_TRY(hipSetDevice(device));
  int rc = run(h_data, stride, len, n, mode, h_initial_arr, initial, h_addrs,
               h_out, device);
  (void)hipSetDevice(prev);
  return rc;
}
