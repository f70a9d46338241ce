// yucsum_host.cpp — host-memory batched entry points
// (yu_csum_batch_host_uniform / _ragged / _iov).
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
// the CPU staging copy of the next slice overlaps all of them. Slices are
// whole packets, about 32 MiB each. Ragged batches ship rebased offsets with
// each slice; scatter-gather (iovec) packets are gathered into the staging
// slot while the previous slices are on the GPU. A batch of at most 4 MiB
// (a tun read burst) skips the copies instead: the kernel reads the pinned
// host memory and writes the results there over PCIe (see `direct`), which
// more than halves the per-call latency. Staging lives in two bounded pools of
// contexts per device (ContextPool: at most YU_HOST_CONTEXTS of each, default 4;
// bulk contexts of 3 slots of at most one slice, burst contexts of one slot for
// the direct calls), checked out for the length of one call and returned:
// concurrent callers share nothing while they hold one, a caller that finds
// every context of its kind in use waits for one, and a burst never waits behind
// bulk batches. Memory therefore
// grows with the number of concurrent calls the pool allows, not with the
// number of OS threads that ever called (a Go caller's goroutines migrate over
// many of them); yu_host_staging_bytes reports it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "yucsum.h"
#include "yucsum_internal.h"

namespace {

constexpr int kSlots = 3;
constexpr uint64_t kSliceBytes = YU_HOST_SLICE_BYTES;  // 32 MiB
// Packets per slice at most: bounds a slot's side arrays (26 bytes of pinned and
// 22 of device memory per packet) as kSliceBytes bounds its packet bytes. Only
// packets under 128 bytes reach it; 256K of 64-byte packets is 16 MiB, still
// hundreds of microseconds of PCIe per slice.
constexpr uint64_t kSlicePkts = YU_HOST_SLICE_PACKETS;  // 256K

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
  uint64_t *h_off = nullptr;
  uint8_t *d_data = nullptr, *d_addrs = nullptr;
  uint16_t *d_init = nullptr, *d_out = nullptr;
  uint64_t *d_off = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t done = nullptr;
  // direct mode: results and a completion flag in coherent pinned memory
  uint16_t *h_outc = nullptr;
  uint32_t *h_flag = nullptr;
  uint32_t seq = 0;
  uint64_t first = 0, cnt = 0, outs = 1;  // outs: results per packet
  bool busy = false, staged_out = false;
};

// Staging bytes of a context reserved for (data_bytes, pk): pinned host and device.
// (the allocations of Ctx::reserve: packet bytes, addrs 8, initial 2, results 4,
// offsets 8, coherent results 4 per packet, one more offset, the 64-byte flag)
constexpr uint64_t pinned_bytes(uint64_t data_bytes, uint64_t pk, int slots = kSlots) {
  return slots * ((data_bytes ? data_bytes : 16) + pk * 8 + pk * 2 + pk * 4 + (pk + 1) * 8 + pk * 4 + 64);
}
constexpr uint64_t device_bytes(uint64_t data_bytes, uint64_t pk, int slots = kSlots) {
  return slots * ((data_bytes ? data_bytes : 16) + pk * 8 + pk * 2 + pk * 4 + (pk + 1) * 8);
}
// The default direct cut-over (bytes of one burst that the kernel reads from
// host memory itself; see `direct` below).
constexpr uint64_t kDirectMax = 4ull << 20;
static_assert(pinned_bytes(kSliceBytes, kSlicePkts) == YU_HOST_CONTEXT_PINNED_MAX, "yucsum.h bound");
static_assert(device_bytes(kSliceBytes, kSlicePkts) == YU_HOST_CONTEXT_DEVICE_MAX, "yucsum.h bound");
static_assert(pinned_bytes(kDirectMax, kSlicePkts, 1) == YU_HOST_BURST_CONTEXT_PINNED_MAX, "yucsum.h bound");
static_assert(device_bytes(kDirectMax, kSlicePkts, 1) == YU_HOST_BURST_CONTEXT_DEVICE_MAX, "yucsum.h bound");
static_assert(kSlots == 3, "yucsum.h bounds assume 3 slots");

struct Ctx {
  int dev = -1;
  int nslots = kSlots;  // 1 for a burst context (the direct path uses slot 0 alone)
  // (atomic: yu_host_staging_bytes reads them while the holder may reserve)
  std::atomic<uint64_t> cap_data{0}, cap_pk{0};
  std::atomic<bool> reserved{false};
  Slot s[kSlots];

  void release() {
    for (int k = 0; k < nslots; ++k) {
      Slot &x = s[k];
      if (x.h_data) (void)hipHostFree(x.h_data);
      if (x.h_addrs) (void)hipHostFree(x.h_addrs);
      if (x.h_init) (void)hipHostFree(x.h_init);
      if (x.h_out) (void)hipHostFree(x.h_out);
      if (x.h_off) (void)hipHostFree(x.h_off);
      if (x.d_data) (void)hipFree(x.d_data);
      if (x.d_addrs) (void)hipFree(x.d_addrs);
      if (x.d_init) (void)hipFree(x.d_init);
      if (x.d_out) (void)hipFree(x.d_out);
      if (x.d_off) (void)hipFree(x.d_off);
      if (x.h_outc) (void)hipHostFree(x.h_outc);
      if (x.h_flag) (void)hipHostFree(x.h_flag);
      if (x.done) (void)hipEventDestroy(x.done);
      if (x.st) (void)hipStreamDestroy(x.st);
      x = Slot();
    }
    cap_data = cap_pk = 0;
    reserved = false;
  }
  ~Ctx() { release_on_device(); }
  // release() with this context's device current (a trim or give-back may run
  // on a thread whose current device is another one); the caller's device is
  // restored.
  void release_on_device() {
    if (dev < 0) return;
    int prev = -1;
    const bool restore = hipGetDevice(&prev) == hipSuccess;
    if (hipSetDevice(dev) != hipSuccess) {
      (void)hipGetLastError();
      return;
    }
    release();
    if (restore && prev != dev) (void)hipSetDevice(prev);
  }

  // Grows the staging to (data_bytes, pk). A failed allocation frees whatever
  // was allocated before it, so a context is either fully reserved (and its
  // caps count it) or holds nothing.
  int reserve(uint64_t data_bytes, uint64_t pk) {
    if (data_bytes <= cap_data && pk <= cap_pk) return YU_OK;
    if (data_bytes < cap_data) data_bytes = cap_data;
    if (pk < cap_pk) pk = cap_pk;
    release();
    const int rc = allocate(data_bytes, pk);
    if (rc) {
      release();
      return rc;
    }
    return YU_OK;
  }

 private:
  // Fault injection for the tests (measurement knob, YU_TUNING=1 only):
  // YU_HOST_FAIL_ALLOC=k makes the k-th staging allocation of the process
  // (1-based, counted over every context) fail once as out of memory.
  static hipError_t inject(hipError_t e) {
    static const long fail_at = [] {
      const char *v = yu::tuning_env("YU_HOST_FAIL_ALLOC");
      return v && *v ? strtol(v, nullptr, 10) : 0L;
    }();
    static std::atomic<long> count{0};
    if (fail_at > 0 && e == hipSuccess && ++count == fail_at) return hipErrorOutOfMemory;
    return e;
  }
#define YU_TRY_ALLOC(expr) YU_TRY(inject(expr))

  int allocate(uint64_t data_bytes, uint64_t pk) {
    // reserved before the first allocation: yu_host_staging_bytes counts a
    // context whose caps are set, and these are set only once all succeeded
    reserved = true;
    for (int k = 0; k < nslots; ++k) {
      Slot &x = s[k];
      YU_TRY(hipStreamCreateWithFlags(&x.st, hipStreamNonBlocking));
      YU_TRY(hipEventCreateWithFlags(&x.done, hipEventDisableTiming));
      YU_TRY_ALLOC(hipHostMalloc((void **)&x.h_data, data_bytes ? data_bytes : 16, 0));
      YU_TRY_ALLOC(hipHostMalloc((void **)&x.h_addrs, pk * 8, 0));
      YU_TRY_ALLOC(hipHostMalloc((void **)&x.h_init, pk * 2, 0));
      // results: up to 2 per packet (YU_MODE_OUTPUTS)
      YU_TRY_ALLOC(hipHostMalloc((void **)&x.h_out, pk * 4, 0));
      YU_TRY_ALLOC(hipHostMalloc((void **)&x.h_off, (pk + 1) * 8, 0));
      YU_TRY_ALLOC(hipHostMalloc((void **)&x.h_outc, pk * 4, hipHostMallocCoherent));
      YU_TRY_ALLOC(hipHostMalloc((void **)&x.h_flag, 64, hipHostMallocCoherent));
      *x.h_flag = 0;
      YU_TRY_ALLOC(hipMalloc((void **)&x.d_data, data_bytes ? data_bytes : 16));
      YU_TRY_ALLOC(hipMalloc((void **)&x.d_addrs, pk * 8));
      YU_TRY_ALLOC(hipMalloc((void **)&x.d_init, pk * 2));
      YU_TRY_ALLOC(hipMalloc((void **)&x.d_out, pk * 4));
      YU_TRY_ALLOC(hipMalloc((void **)&x.d_off, (pk + 1) * 8));
    }
    cap_data = data_bytes;
    cap_pk = pk;
    return YU_OK;
  }
#undef YU_TRY_ALLOC
};

// Upper bound on the staging contexts of one device (YU_HOST_CONTEXTS, 1..64,
// default 4): a product setting, like the reference's tundev.BufConfig
// (link/tundev/tundev.go:20), not a measurement knob, so it is read without the
// YU_TUNING gate.
int host_contexts() {
  static const int v = [] {
    const char *e = getenv("YU_HOST_CONTEXTS");
    char *end = nullptr;
    const long k = e && *e ? strtol(e, &end, 10) : 4;
    if (e && *e && *end) return 4;  // not a number: the default
    return (int)(k < 1 ? 1 : (k > 64 ? 64 : k));
  }();
  return v;
}

// The bounded context pool of one device. Contexts are created lazily, up to
// host_contexts(), and live for the process (never destroyed at exit, when the
// HIP runtime may already be gone); an idle one is lent to the next caller.
class ContextPool {
 public:
  // slots: kSlots (bulk pool) or 1 (burst pool)
  Ctx *acquire(int dev, int slots) {
    std::unique_lock<std::mutex> l(m_);
    cv_.wait(l, [&] { return !idle_.empty() || (int)all_.size() < host_contexts(); });
    Ctx *c;
    if (!idle_.empty()) {
      c = idle_.back();
      idle_.pop_back();
    } else {
      all_.push_back(new Ctx());
      c = all_.back();
      c->dev = dev;
      c->nslots = slots;
    }
    return c;
  }
  // A context that grew past its standard size (a packet longer than
  // kSliceBytes is a slice of its own; a burst context that served a fallback or
  // a tuned, larger direct cut-over) gives that memory back here, so the pools
  // keep at most host_contexts() x their standard budgets between calls.
  void give_back(Ctx *c) {
    const uint64_t cap = c->nslots == kSlots ? kSliceBytes : kDirectMax;
    if (c->cap_data > cap || c->cap_pk > kSlicePkts) c->release_on_device();
    {
      std::lock_guard<std::mutex> l(m_);
      idle_.push_back(c);
    }
    cv_.notify_one();
  }
  // Staging held right now by this device's contexts (idle and lent).
  void held(uint64_t &pinned, uint64_t &dev) {
    std::lock_guard<std::mutex> l(m_);
    pinned = dev = 0;
    for (Ctx *c : all_) {
      if (!c->reserved) continue;
      pinned += pinned_bytes(c->cap_data, c->cap_pk, c->nslots);
      dev += device_bytes(c->cap_data, c->cap_pk, c->nslots);
    }
  }
  // Frees the staging of every idle context (lent ones are left alone). Each
  // context is taken out of the idle list and freed outside the lock (hipFree
  // and hipHostFree may wait on the device), so a concurrent acquire() can take
  // any other idle context meanwhile; it is put back and a waiter woken after.
  void trim() {
    std::vector<Ctx *> todo;
    {
      std::lock_guard<std::mutex> l(m_);
      for (Ctx *c : idle_)
        if (c->reserved) todo.push_back(c);
    }
    for (Ctx *c : todo) {
      {
        std::lock_guard<std::mutex> l(m_);
        auto it = std::find(idle_.begin(), idle_.end(), c);
        if (it == idle_.end()) continue;  // lent meanwhile: its holder keeps it
        idle_.erase(it);
      }
      c->release_on_device();
      {
        std::lock_guard<std::mutex> l(m_);
        idle_.push_back(c);
      }
      cv_.notify_one();
    }
  }
 private:
  std::mutex m_;
  std::condition_variable cv_;
  std::vector<Ctx *> all_, idle_;
};

// Two pools per device: bulk contexts (3 slots, any call) and burst contexts (1
// slot, calls that take the direct path), so a tun burst never waits behind
// bulk batches that hold every bulk context.
enum PoolKind { kBulk = 0, kBurst = 1 };

ContextPool &pool_of(int device, int kind) {
  static ContextPool *pools = new ContextPool[2 * 64];  // process lifetime
  return pools[2 * device + kind];
}

// Staging copies of pageable input. One thread's memcpy into pinned memory
// runs at roughly half the PCIe rate, so a 32 MiB slice is split across a small
// pool of persistent threads plus the caller. The pool serves one staging copy
// at a time; a concurrent caller (another device's worker) copies on its own
// thread instead of waiting. YU_HOST_COPY_THREADS sets the pool size (default
// 7 helpers; 0 disables it).
class CopyPool {
 public:
  static CopyPool &get() {
    static CopyPool *p = new CopyPool();  // process lifetime: the helpers are detached
    return *p;
  }
  // fn(i) for every i in [0, parts), on the helpers and the calling thread.
  // Returns false (nothing run) when the pool is busy or empty.
  bool run(int parts, const std::function<void(int)> &fn) {
    if (nthreads_ == 0 || parts < 2) return false;
    std::unique_lock<std::mutex> busy(run_m_, std::try_to_lock);
    if (!busy.owns_lock()) return false;
    {
      std::lock_guard<std::mutex> l(m_);
      job_ = &fn;
      parts_ = parts;
      next_ = 0;
      done_ = 0;
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> l(m_);
    done_cv_.wait(l, [&] { return done_ == parts_; });
    job_ = nullptr;
    return true;
  }
  int threads() const { return nthreads_; }

 private:
  CopyPool() {
    const char *e = yu::tuning_env("YU_HOST_COPY_THREADS");
    nthreads_ = e && *e ? atoi(e) : 7;
    if (nthreads_ < 0) nthreads_ = 0;
    if (nthreads_ > 64) nthreads_ = 64;
    for (int i = 0; i < nthreads_; ++i) std::thread([this] { loop(); }).detach();
  }
  // Claims parts of the current job until none are left.
  void work() {
    for (;;) {
      int i;
      const std::function<void(int)> *f;
      {
        std::lock_guard<std::mutex> l(m_);
        if (!job_ || next_ >= parts_) return;
        i = next_++;
        f = job_;
      }
      (*f)(i);
      std::lock_guard<std::mutex> l(m_);
      if (++done_ == parts_) done_cv_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return gen_ != seen; });
        seen = gen_;
      }
      work();
    }
  }
  int nthreads_ = 0;
  std::mutex run_m_, m_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)> *job_ = nullptr;
  int parts_ = 0, next_ = 0, done_ = 0;
  uint64_t gen_ = 0;
};

constexpr uint64_t kParCopyMin = 1ull << 20;  // below this one memcpy is faster

void stage_copy(uint8_t *dst, const uint8_t *src, uint64_t n) {
  CopyPool &pool = CopyPool::get();
  if (n >= 2 * kParCopyMin) {
    const uint64_t parts = std::min<uint64_t>((uint64_t)pool.threads() + 1, n / kParCopyMin);
    const uint64_t chunk = ((n + parts - 1) / parts + 63) & ~63ull;
    if (pool.run((int)parts, [&](int i) {
          const uint64_t a = (uint64_t)i * chunk;
          if (a < n) memcpy(dst + a, src + a, std::min(chunk, n - a));
        }))
      return;
  }
  memcpy(dst, src, n);
}

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
  if (x.staged_out) memcpy(h_out + x.first * x.outs, x.h_out, x.cnt * 2 * x.outs);
  x.busy = false;
  return YU_OK;
}

// A context of `device` for the length of one call (RAII: returned to the pool
// on every exit path).
class Lease {
 public:
  Lease(int device, int kind)
      : device_(device), kind_(kind), c_(pool_of(device, kind).acquire(device, kind == kBurst ? 1 : kSlots)) {
    // A previous call that failed midway may have left slices in flight:
    // drain them without copying (their h_out belonged to that call).
    for (Slot &x : c_->s) {
      if (x.busy) (void)hipEventSynchronize(x.done);
      x.busy = false;
    }
  }
  ~Lease() { pool_of(device_, kind_).give_back(c_); }
  Lease(const Lease &) = delete;
  Lease &operator=(const Lease &) = delete;
  Ctx &ctx() { return *c_; }

 private:
  int device_, kind_;
  Ctx *c_;
};

// Small batches (a tun read burst) go "direct": the kernel reads the pinned
// host bytes and side arrays and writes the results over PCIe itself — one
// launch and one synchronisation instead of H2D copies, a launch and a D2H
// copy, whose fixed latencies (not bandwidth) dominate a batch this size.
// Pageable inputs are first copied into the slot's pinned staging, as on the
// pipelined path. Measured per call (pinned 1500-B TCP segments, round 1):
// 64 packets 32.5 -> 20-21 us, 1024 packets 64.6 -> 50.3 us, 8192 packets
// (12 MB) 258 -> 289 us, so the cut-over is 4 MiB. YU_HOST_DIRECT_MAX (bytes,
// measurement knob) moves it; 0 disables direct mode.
constexpr int kNoDirect = 1;  // not an error: take the pipelined path

uint64_t direct_max() {
  static const uint64_t v = [] {
    const char *e = yu::tuning_env("YU_HOST_DIRECT_MAX");
    return e && *e ? strtoull(e, nullptr, 10) : kDirectMax;
  }();
  return v;
}

template <class T>
bool dev_view(const T *h, T **d) {
  void *p = nullptr;
  if (hipHostGetDevicePointer(&p, (void *)h, 0) != hipSuccess || !p) {
    (void)hipGetLastError();
    return false;
  }
  *d = (T *)p;
  return true;
}

// Spin until the slot's flag reaches seq. A kernel fault (or a stalled box)
// never raises it: after ~0.25 s of spinning the stream is synchronised, which
// reports the error.
int wait_flag(Slot &x, uint32_t seq) {
  for (uint32_t i = 0; i < (1u << 22); ++i) {
    if (__atomic_load_n(x.h_flag, __ATOMIC_ACQUIRE) == seq) return YU_OK;
    __builtin_ia32_pause();
  }
  YU_TRY(hipStreamSynchronize(x.st));
  return __atomic_load_n(x.h_flag, __ATOMIC_ACQUIRE) == seq ? YU_OK : YU_EHIP_BASE;
}

template <class Layout>
int direct(Slot &x, const Layout &L, uint64_t n, const uint16_t *h_init,
           const uint8_t *h_addrs, uint16_t *h_out) {
  const uint8_t *src = L.stage(x, 0, n);  // the caller's pinned bytes or the slot's staging
  uint8_t *d = nullptr, *da = nullptr;
  uint64_t *doff = nullptr;
  uint16_t *di = nullptr, *dout = nullptr;
  if (L.bytes(0, n) && !dev_view(src, &d)) return kNoDirect;
  if (!d && !dev_view(x.h_data, &d)) return kNoDirect;  // empty packets: any valid base
  if (L.ragged() && !dev_view(x.h_off, &doff)) return kNoDirect;
  if (h_init) {
    memcpy(x.h_init, h_init, n * 2);
    if (!dev_view(x.h_init, &di)) return kNoDirect;
  }
  if (h_addrs) {
    memcpy(x.h_addrs, h_addrs, n * 8);
    if (!dev_view(x.h_addrs, &da)) return kNoDirect;
  }
  uint32_t *dflag = nullptr;
  if (!dev_view(x.h_outc, &dout) || !dev_view(x.h_flag, &dflag)) return kNoDirect;
  int rc = L.launch(d, doff, n, di, da, dout, x.st);
  if (rc) return rc;
  // Completion by polling a flag the GPU stores after the kernel, instead of
  // hipStreamSynchronize: 3-4 us less per call (tools/host_lat.cpp). Results
  // and flag live in coherent (uncached) pinned memory, written in order.
  const uint32_t seq = ++x.seq;
  rc = yu_internal_signal(dflag, seq, x.st);
  if (rc) return rc;
  rc = wait_flag(x, seq);
  if (rc) return rc;
  memcpy(h_out, x.h_outc, n * 2 * YU_MODE_OUTPUTS(L.mode));
  return YU_OK;
}

// The slice pipeline shared by the layouts. A Layout says how many packets
// the slice starting at `first` holds (byte-bounded), how many bytes they
// span, how to stage them (returning the host pointer the H2D copy reads:
// the caller's pinned buffer or the slot's staging), and how to launch.
template <class Layout>
int run_slices(Ctx &c, const Layout &L, uint64_t n, const uint16_t *h_init,
               const uint8_t *h_addrs, uint16_t *h_out, bool pin_out);

// One host batch on the current device: its slices' geometry first (no context
// needed), then a context from the burst pool when the batch takes the direct
// path (one slice of at most direct_max() bytes) or from the bulk pool otherwise.
template <class Layout>
int pipeline(int device, const Layout &L, uint64_t n, const uint16_t *h_init,
             const uint8_t *h_addrs, uint16_t *h_out) {
  // capacity: the largest slice of this batch
  uint64_t max_b = 0, max_pk = 0;
  for (uint64_t first = 0; first < n;) {
    const uint64_t cnt = L.count(first);
    const uint64_t b = L.bytes(first, cnt);
    if (b > max_b) max_b = b;
    if (cnt > max_pk) max_pk = cnt;
    first += cnt;
  }
  const bool burst = max_pk == n && max_b <= direct_max();
  Lease lease(device, burst ? kBurst : kBulk);
  Ctx &c = lease.ctx();
  int rc = c.reserve(max_b, max_pk);
  if (rc) return rc;
  rc = kNoDirect;
  if (burst) rc = direct(c.s[0], L, n, h_init, h_addrs, h_out);
  // (a burst whose memory cannot be mapped for the kernel falls back to the copies,
  // through its context's one slot)
  if (rc == kNoDirect) rc = run_slices(c, L, n, h_init, h_addrs, h_out, is_pinned(h_out));
  if (rc) {
    // A failed call returns with no transfer still aimed at the caller's
    // buffers: every slot's stream is drained before the error goes back (a
    // pinned input is read, and a pinned h_out written, by the copies
    // themselves, including those of a slice that failed halfway).
    for (int k = 0; k < c.nslots; ++k) {
      Slot &x = c.s[k];
      if (x.st) (void)hipStreamSynchronize(x.st);
      x.busy = false;
    }
    (void)hipGetLastError();
  }
  return rc;
}

template <class Layout>
int run_slices(Ctx &c, const Layout &L, uint64_t n, const uint16_t *h_init,
               const uint8_t *h_addrs, uint16_t *h_out, bool pin_out) {
  int rc = YU_OK;
  const uint64_t outs = YU_MODE_OUTPUTS(L.mode);  // results per packet
  uint64_t k = 0;                                 // slice counter: slot k % nslots
  for (uint64_t first = 0; first < n; ++k) {
    Slot &x = c.s[k % (uint64_t)c.nslots];
    rc = finish(x, h_out);
    if (rc) return rc;
    const uint64_t cnt = L.count(first);
    const uint64_t bytes = L.bytes(first, cnt);
    const uint8_t *src = L.stage(x, first, cnt);
    if (bytes) YU_TRY(hipMemcpyAsync(x.d_data, src, bytes, hipMemcpyHostToDevice, x.st));
    if (L.ragged())
      YU_TRY(hipMemcpyAsync(x.d_off, x.h_off, (cnt + 1) * 8, hipMemcpyHostToDevice, x.st));
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
    rc = L.launch(x.d_data, x.d_off, cnt, d_init, d_addrs, x.d_out, x.st);
    if (rc) return rc;
    x.staged_out = !pin_out;
    YU_TRY(hipMemcpyAsync(pin_out ? h_out + first * outs : x.h_out, x.d_out, cnt * 2 * outs,
                          hipMemcpyDeviceToHost, x.st));
    x.outs = outs;
    YU_TRY(hipEventRecord(x.done, x.st));
    x.first = first;
    x.cnt = cnt;
    x.busy = true;
    first += cnt;
  }
  for (int j = 0; j < c.nslots; ++j) {
    rc = finish(c.s[j], h_out);
    if (rc) return rc;
  }
  return YU_OK;
}

// packet i = data[i*stride, i*stride + len)
struct UniformLayout {
  const uint8_t *h_data;
  uint64_t stride, n, slice;
  uint32_t len;
  int mode;
  uint16_t initial;
  bool pin_in;
  bool ragged() const { return false; }
  uint64_t count(uint64_t first) const { return n - first < slice ? n - first : slice; }
  uint64_t bytes(uint64_t, uint64_t cnt) const { return (cnt - 1) * stride + len; }
  const uint8_t *stage(Slot &x, uint64_t first, uint64_t cnt) const {
    const uint8_t *src = h_data + first * stride;
    const uint64_t b = bytes(first, cnt);
    if (pin_in || !b) return src;
    stage_copy(x.h_data, src, b);
    return x.h_data;
  }
  int launch(const uint8_t *d, const uint64_t *, uint64_t cnt, const uint16_t *d_init,
             const uint8_t *d_addrs, uint16_t *d_out, hipStream_t st) const {
    return yu_csum_batch_uniform(d, stride, len, cnt, mode, d_init, initial, d_addrs, d_out, st);
  }
};

// Slices of whole packets, each up to kSliceBytes (a longer packet is a
// slice of its own); `span(i)` = bytes of packet i.
template <class Span>
uint64_t byte_slice(uint64_t first, uint64_t n, const Span &span) {
  uint64_t cnt = 0, b = 0;
  while (first + cnt < n && cnt < kSlicePkts) {
    const uint64_t l = span(first + cnt);
    if (cnt && b + l > kSliceBytes) break;
    b += l;
    ++cnt;
  }
  return cnt;
}

// packet i = data[off[i], off[i+1]) (tun burst, back to back)
struct RaggedLayout {
  const uint8_t *h_data;
  const uint64_t *off;
  uint64_t n;
  int mode;
  uint16_t initial;
  bool pin_in;
  bool ragged() const { return true; }
  uint64_t count(uint64_t first) const {
    return byte_slice(first, n, [&](uint64_t i) { return off[i + 1] - off[i]; });
  }
  uint64_t bytes(uint64_t first, uint64_t cnt) const { return off[first + cnt] - off[first]; }
  const uint8_t *stage(Slot &x, uint64_t first, uint64_t cnt) const {
    const uint64_t o0 = off[first];
    for (uint64_t i = 0; i <= cnt; ++i) x.h_off[i] = off[first + i] - o0;
    const uint64_t b = bytes(first, cnt);
    if (pin_in || !b) return h_data + o0;
    stage_copy(x.h_data, h_data + o0, b);
    return x.h_data;
  }
  int launch(const uint8_t *d, const uint64_t *d_off, uint64_t cnt, const uint16_t *d_init,
             const uint8_t *d_addrs, uint16_t *d_out, hipStream_t st) const {
    return yu_csum_batch_ragged(d, d_off, cnt, mode, d_init, initial, d_addrs, d_out, st);
  }
};

// packet i = iov[first_iov[i]] ‖ ... ‖ iov[first_iov[i+1] - 1], gathered
// into the staging slot (the tun endpoint's readv into 4 views,
// link/tundev/tundev.go:116-125, buffer/view.go:37-46)
struct IovLayout {
  const yu_iovec *iov;
  const uint64_t *first_iov;
  uint64_t n;
  int mode;
  uint16_t initial;
  bool ragged() const { return true; }
  uint64_t plen(uint64_t i) const {
    uint64_t l = 0;
    for (uint64_t v = first_iov[i]; v < first_iov[i + 1]; ++v) l += iov[v].len;
    return l;
  }
  uint64_t count(uint64_t first) const {
    return byte_slice(first, n, [&](uint64_t i) { return plen(i); });
  }
  uint64_t bytes(uint64_t first, uint64_t cnt) const {
    uint64_t b = 0;
    for (uint64_t i = first; i < first + cnt; ++i) b += plen(i);
    return b;
  }
  const uint8_t *stage(Slot &x, uint64_t first, uint64_t cnt) const {
    uint64_t o = 0;
    for (uint64_t i = 0; i < cnt; ++i) {
      x.h_off[i] = o;
      o += plen(first + i);
    }
    x.h_off[cnt] = o;
    // gather packets [a, b) of the slice into their staging offsets
    auto gather = [&](uint64_t a, uint64_t b) {
      for (uint64_t i = a; i < b; ++i) {
        uint64_t d = x.h_off[i];
        for (uint64_t v = first_iov[first + i]; v < first_iov[first + i + 1]; ++v) {
          if (iov[v].len) memcpy(x.h_data + d, iov[v].base, iov[v].len);
          d += iov[v].len;
        }
      }
    };
    CopyPool &pool = CopyPool::get();
    const uint64_t parts = std::min<uint64_t>((uint64_t)pool.threads() + 1, o / kParCopyMin);
    if (parts >= 2 && cnt >= parts) {
      const uint64_t per = (cnt + parts - 1) / parts;
      if (pool.run((int)parts, [&](int i) {
            const uint64_t a = (uint64_t)i * per;
            gather(std::min(a, cnt), std::min(a + per, cnt));
          }))
        return x.h_data;
    }
    gather(0, cnt);
    return x.h_data;
  }
  int launch(const uint8_t *d, const uint64_t *d_off, uint64_t cnt, const uint16_t *d_init,
             const uint8_t *d_addrs, uint16_t *d_out, hipStream_t st) const {
    return yu_csum_batch_ragged(d, d_off, cnt, mode, d_init, initial, d_addrs, d_out, st);
  }
};

// Device selection around one call; the caller's current device is restored.
template <class F>
int on_device(int device, F &&f) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return YU_ENODEV;
  if (device < 0 || device >= ndev || device >= 64) return YU_ENODEV;
  int prev = 0;
  YU_TRY(hipGetDevice(&prev));
  YU_TRY(hipSetDevice(device));
  const int rc = f();
  (void)hipSetDevice(prev);
  return rc;
}

bool bad_mode(int mode) { return mode < 0 || mode >= YU_MODE_COUNT; }

// A uniform batch [data, data + (n-1)*stride + len) that would wrap the
// address space (a nonsense stride or count) is rejected before any copy.
bool span_wraps(const uint8_t *data, uint64_t stride, uint32_t len, uint64_t n) {
  return n > 1 && stride > (UINT64_MAX - (uint64_t)(uintptr_t)data - len) / (n - 1);
}

// Host offsets are checked here, unlike the device call's: non-decreasing,
// every packet within the mode's length limit.
int check_offsets(const uint64_t *off, uint64_t n, int mode) {
  const uint64_t cap = mode == YU_MODE_RAW ? YU_MAX_RAW_LEN : YU_MAX_TRANSPORT_LEN;
  for (uint64_t i = 0; i < n; ++i) {
    if (off[i + 1] < off[i]) return YU_EINVAL;        // EINVAL:offsets
    if (off[i + 1] - off[i] > cap) return YU_EINVAL;  // EINVAL:len-transport / len-raw
  }
  return YU_OK;
}

// Scatter-gather packet index: non-decreasing view ranges, no NULL view with
// bytes, every packet within the mode's length limit.
int check_iov(const yu_iovec *iov, const uint64_t *first_iov, uint64_t n, int mode) {
  const uint64_t cap = mode == YU_MODE_RAW ? YU_MAX_RAW_LEN : YU_MAX_TRANSPORT_LEN;
  for (uint64_t i = 0; i < n; ++i) {
    if (first_iov[i + 1] < first_iov[i]) return YU_EINVAL;  // EINVAL:offsets
    uint64_t l = 0;
    for (uint64_t v = first_iov[i]; v < first_iov[i + 1]; ++v) {
      if (!iov[v].base && iov[v].len) return YU_EINVAL;  // EINVAL:iov-view
      // l <= cap: no wrap, even for huge views
      if (iov[v].len > cap - l) return YU_EINVAL;  // EINVAL:len-transport / len-raw
      l += iov[v].len;
    }
  }
  return YU_OK;
}

// Multi-GPU host path: the batch is cut into one contiguous
// shard per listed device and each shard runs the single-device pipeline on
// that device's persistent worker thread, so every GPU's PCIe link, copy
// engines and staging slots work at once. Packets are independent: there is
// no exchange, each shard writes its own range of h_out. The workers live for
// the process (their thread-local staging contexts are reused across calls);
// one worker per device serialises the shards concurrent callers give it.
class Worker {
 public:
  Worker() { std::thread([this] { loop(); }).detach(); }
  void post(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> l(m_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return !q_.empty(); });
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
};

Worker &worker(int device) {
  static std::mutex gm;
  static Worker *w[64];  // process lifetime, never freed (threads are detached)
  std::lock_guard<std::mutex> l(gm);
  if (!w[device]) w[device] = new Worker();
  return *w[device];
}

bool bad_devices(const int *devices, int ndev) { return !devices || ndev < 1 || ndev > 64; }

int check_devices(const int *devices, int ndev) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return YU_ENODEV;
  for (int i = 0; i < ndev; ++i)
    if (devices[i] < 0 || devices[i] >= count || devices[i] >= 64) return YU_ENODEV;
  return YU_OK;
}

// Runs shard(i, first, cnt) for the shards [bounds[i], bounds[i+1]) on
// worker(devices[i]) and waits for all of them; returns the first failure.
int fan_out(const int *devices, int ndev, const std::vector<uint64_t> &bounds,
            const std::function<int(int, uint64_t, uint64_t)> &shard) {
  std::mutex m;
  std::condition_variable cv;
  int pending = 0, rc = YU_OK;
  for (int i = 0; i < ndev; ++i) {
    const uint64_t a = bounds[i], b = bounds[i + 1];
    if (a == b) continue;
    {
      std::lock_guard<std::mutex> l(m);
      ++pending;
    }
    worker(devices[i]).post([&, i, a, b] {
      const int r = shard(i, a, b - a);
      std::lock_guard<std::mutex> l(m);
      if (r != YU_OK && rc == YU_OK) rc = r;
      if (--pending == 0) cv.notify_all();
    });
  }
  std::unique_lock<std::mutex> l(m);
  cv.wait(l, [&] { return pending == 0; });
  return rc;
}

// Even packet counts (uniform, iovec).
std::vector<uint64_t> even_bounds(uint64_t n, int ndev) {
  std::vector<uint64_t> b(ndev + 1);
  for (int i = 0; i <= ndev; ++i) b[i] = (uint64_t)((unsigned __int128)n * i / ndev);
  return b;
}

// Packet boundaries closest below an even split of the bytes (ragged), as
// yustack_amd/shard.py does for the device-resident bench.
std::vector<uint64_t> byte_bounds(const uint64_t *off, uint64_t n, int ndev) {
  std::vector<uint64_t> b(ndev + 1);
  const uint64_t o0 = off[0], tot = off[n] - off[0];
  b[0] = 0;
  b[ndev] = n;
  for (int i = 1; i < ndev; ++i) {
    const uint64_t target = o0 + (uint64_t)((unsigned __int128)tot * i / ndev);
    uint64_t k = (uint64_t)(std::lower_bound(off, off + n + 1, target) - off);
    if (k > n) k = n;
    b[i] = std::max(k, b[i - 1]);
  }
  return b;
}

}  // namespace

extern "C" int yu_csum_batch_host_uniform(const uint8_t *h_data,
                                          uint64_t stride, uint32_t len,
                                          uint64_t n, int mode,
                                          const uint16_t *h_initial_arr,
                                          uint16_t initial,
                                          const uint8_t *h_addrs,
                                          uint16_t *h_out, int device) {
  if (bad_mode(mode)) return YU_EINVAL;  // EINVAL:mode
  if (n == 0) return YU_OK;              // (an empty batch may pass a NULL h_out)
  if (!h_out) return YU_EINVAL;          // EINVAL:out
  if (!h_data && len) return YU_EINVAL;                                      // EINVAL:data
  if (mode != YU_MODE_RAW && len > YU_MAX_TRANSPORT_LEN) return YU_EINVAL;  // EINVAL:len-transport
  if (len > YU_MAX_RAW_LEN) return YU_EINVAL;                                // EINVAL:len-raw
  if (span_wraps(h_data, stride, len, n)) return YU_EINVAL;                  // EINVAL:span
  return on_device(device, [&] {
    const uint64_t pstride = stride ? stride : 1;
    uint64_t slice = kSliceBytes / pstride;
    if (slice > kSlicePkts) slice = kSlicePkts;
    if (slice < 1) slice = 1;
    if (slice > n) slice = n;
    UniformLayout L{h_data, stride, n, slice, len, mode, initial, is_pinned(h_data)};
    return pipeline(device, L, n, h_initial_arr, h_addrs, h_out);
  });
}

extern "C" int yu_csum_batch_host_ragged(const uint8_t *h_data,
                                         const uint64_t *h_offsets, uint64_t n,
                                         int mode, const uint16_t *h_initial_arr,
                                         uint16_t initial,
                                         const uint8_t *h_addrs,
                                         uint16_t *h_out, int device) {
  if (bad_mode(mode)) return YU_EINVAL;  // EINVAL:mode
  if (n == 0) return YU_OK;              // (an empty batch may pass a NULL h_out)
  if (!h_out) return YU_EINVAL;          // EINVAL:out
  if (!h_offsets) return YU_EINVAL;                                   // EINVAL:offsets
  if (!h_data && h_offsets[n] != h_offsets[0]) return YU_EINVAL;     // EINVAL:data
  if (int rc = check_offsets(h_offsets, n, mode)) return rc;
  return on_device(device, [&] {
    RaggedLayout L{h_data, h_offsets, n, mode, initial, is_pinned(h_data)};
    return pipeline(device, L, n, h_initial_arr, h_addrs, h_out);
  });
}

extern "C" int yu_csum_batch_host_iov(const yu_iovec *iov,
                                      const uint64_t *first_iov, uint64_t n,
                                      int mode, const uint16_t *h_initial_arr,
                                      uint16_t initial, const uint8_t *h_addrs,
                                      uint16_t *h_out, int device) {
  if (bad_mode(mode)) return YU_EINVAL;  // EINVAL:mode
  if (n == 0) return YU_OK;              // (an empty batch may pass a NULL h_out)
  if (!h_out) return YU_EINVAL;          // EINVAL:out
  if (!first_iov) return YU_EINVAL;                                   // EINVAL:offsets
  if (!iov && first_iov[n] != first_iov[0]) return YU_EINVAL;        // EINVAL:iov-view
  if (int rc = check_iov(iov, first_iov, n, mode)) return rc;
  return on_device(device, [&] {
    IovLayout L{iov, first_iov, n, mode, initial};
    return pipeline(device, L, n, h_initial_arr, h_addrs, h_out);
  });
}

extern "C" int yu_csum_batch_host_uniform_multi(const uint8_t *h_data, uint64_t stride,
                                                uint32_t len, uint64_t n, int mode,
                                                const uint16_t *h_initial_arr,
                                                uint16_t initial, const uint8_t *h_addrs,
                                                uint16_t *h_out, const int *devices,
                                                int ndev) {
  if (bad_mode(mode)) return YU_EINVAL;                // EINVAL:mode
  if (bad_devices(devices, ndev)) return YU_EINVAL;    // EINVAL:devices
  if (n == 0) return YU_OK;                            // (h_out may be NULL then)
  if (!h_out) return YU_EINVAL;                        // EINVAL:out
  if (!h_data && len) return YU_EINVAL;                                      // EINVAL:data
  if (mode != YU_MODE_RAW && len > YU_MAX_TRANSPORT_LEN) return YU_EINVAL;  // EINVAL:len-transport
  if (len > YU_MAX_RAW_LEN) return YU_EINVAL;                                // EINVAL:len-raw
  if (span_wraps(h_data, stride, len, n)) return YU_EINVAL;                  // EINVAL:span
  if (int rc = check_devices(devices, ndev)) return rc;
  return fan_out(devices, ndev, even_bounds(n, ndev), [&](int i, uint64_t a, uint64_t cnt) {
    return yu_csum_batch_host_uniform(h_data ? h_data + a * stride : nullptr, stride, len, cnt,
                                      mode, h_initial_arr ? h_initial_arr + a : nullptr, initial,
                                      h_addrs ? h_addrs + 8 * a : nullptr, h_out + a * YU_MODE_OUTPUTS(mode), devices[i]);
  });
}

extern "C" int yu_csum_batch_host_ragged_multi(const uint8_t *h_data,
                                               const uint64_t *h_offsets, uint64_t n,
                                               int mode, const uint16_t *h_initial_arr,
                                               uint16_t initial, const uint8_t *h_addrs,
                                               uint16_t *h_out, const int *devices,
                                               int ndev) {
  if (bad_mode(mode)) return YU_EINVAL;                // EINVAL:mode
  if (bad_devices(devices, ndev)) return YU_EINVAL;    // EINVAL:devices
  if (n == 0) return YU_OK;                            // (h_out may be NULL then)
  if (!h_out) return YU_EINVAL;                        // EINVAL:out
  if (!h_offsets) return YU_EINVAL;                                   // EINVAL:offsets
  if (!h_data && h_offsets[n] != h_offsets[0]) return YU_EINVAL;     // EINVAL:data
  if (int rc = check_offsets(h_offsets, n, mode)) return rc;
  if (int rc = check_devices(devices, ndev)) return rc;
  return fan_out(devices, ndev, byte_bounds(h_offsets, n, ndev),
                 [&](int i, uint64_t a, uint64_t cnt) {
                   return yu_csum_batch_host_ragged(
                       h_data, h_offsets + a, cnt, mode,
                       h_initial_arr ? h_initial_arr + a : nullptr, initial,
                       h_addrs ? h_addrs + 8 * a : nullptr, h_out + a * YU_MODE_OUTPUTS(mode), devices[i]);
                 });
}

extern "C" int yu_csum_batch_host_iov_multi(const yu_iovec *iov, const uint64_t *first_iov,
                                            uint64_t n, int mode,
                                            const uint16_t *h_initial_arr, uint16_t initial,
                                            const uint8_t *h_addrs, uint16_t *h_out,
                                            const int *devices, int ndev) {
  if (bad_mode(mode)) return YU_EINVAL;                // EINVAL:mode
  if (bad_devices(devices, ndev)) return YU_EINVAL;    // EINVAL:devices
  if (n == 0) return YU_OK;                            // (h_out may be NULL then)
  if (!h_out) return YU_EINVAL;                        // EINVAL:out
  if (!first_iov) return YU_EINVAL;                                   // EINVAL:offsets
  if (!iov && first_iov[n] != first_iov[0]) return YU_EINVAL;        // EINVAL:iov-view
  if (int rc = check_iov(iov, first_iov, n, mode)) return rc;
  if (int rc = check_devices(devices, ndev)) return rc;
  return fan_out(devices, ndev, even_bounds(n, ndev), [&](int i, uint64_t a, uint64_t cnt) {
    return yu_csum_batch_host_iov(iov, first_iov + a, cnt, mode,
                                  h_initial_arr ? h_initial_arr + a : nullptr, initial,
                                  h_addrs ? h_addrs + 8 * a : nullptr, h_out + a * YU_MODE_OUTPUTS(mode), devices[i]);
  });
}

extern "C" uint64_t yu_host_staging_bytes(int device, uint64_t *dev_bytes) {
  uint64_t pinned = 0, dev = 0;
  for (int kind : {kBulk, kBurst}) {
    uint64_t p = 0, d = 0;
    if (device >= 0 && device < 64) pool_of(device, kind).held(p, d);
    pinned += p;
    dev += d;
  }
  if (dev_bytes) *dev_bytes = dev;
  return pinned;
}

extern "C" int yu_host_contexts(void) { return host_contexts(); }

extern "C" const char *yu_hip_runtime_path(void) {
  // The address of an imported function, taken in this library, is the
  // definition its calls go to (through the GOT), interposition included.
  Dl_info info;
  if (dladdr((void *)&hipGetDevice, &info) == 0 || !info.dli_fname) return nullptr;
  return info.dli_fname;
}

extern "C" int yu_host_staging_trim(int device) {
  if (device < 0 || device >= 64) return YU_ENODEV;
  int prev = 0;
  const bool restore = hipGetDevice(&prev) == hipSuccess;
  if (hipSetDevice(device) != hipSuccess) {
    (void)hipGetLastError();
    return YU_ENODEV;
  }
  pool_of(device, kBulk).trim();
  pool_of(device, kBurst).trim();
  if (restore) (void)hipSetDevice(prev);
  return YU_OK;
}

// ---------------------------------------------------------------------
// Host-memory field writer (SURVEY.md §8f row 3 for packets in host memory):
// the batch runs through the host path above, then the CPU stores each TX
// result big-endian into the packet's checksum field (UDP.SetChecksum
// header/udp.go:60-62, TCP.SetChecksum header/tcp.go:156-158,
// IPv4.SetChecksum header/ipv4.go:165-167, ICMPv4.SetChecksum
// header/icmpv4.go:46-48). The results cross PCIe as 2 bytes per packet
// either way; writing the fields on the GPU would send every packet back.
// The same rule as the device writer decides when a field is stored: it must
// lie inside the packet (IPv4: inside min(len, IHL*4)).
// ---------------------------------------------------------------------
namespace {

using yu::l4_field;  // the kernels' protocol tables (yucsum_internal.h)
using yu::l4_min;
using yu::mode_field;

bool tx_mode(int m) { return yu::mode_fills(m); }

// Byte k of packet i, through a layout's accessor (nullptr past the packet).
// set(i) writes packet i's field; the packets are split over the copy pool.
template <class At>
void put_field(const At &at, uint64_t i, uint32_t f, uint16_t v) {
  uint8_t *hi = at(i, f), *lo = at(i, f + 1);
  if (!hi || !lo) return;
  *hi = (uint8_t)(v >> 8);
  *lo = (uint8_t)v;
}

// TX_DATAGRAM: both fields of datagram i where the device defined them
// (include/yucsum.h): the contract 20 <= HeaderLength() <= TotalLength() <=
// len read from the bytes, the transport field when the protocol has one and
// the segment holds its header — the rule the kernels apply.
template <class At>
void put_datagram_fields(const At &at, uint64_t i, const uint16_t *res) {
  const uint8_t *b0 = at(i, 0), *b2 = at(i, 2), *b3 = at(i, 3), *b9 = at(i, 9);
  if (!at(i, 19)) return;  // shorter than 20 bytes
  const uint32_t hl = (uint32_t)(*b0 & 0xFu) * 4u, tl = (uint32_t)*b2 << 8 | *b3;
  if (hl < 20u || hl > tl || !at(i, tl - 1u)) return;
  put_field(at, i, 10, res[2 * i]);
  const uint32_t proto = *b9;
  const uint32_t fo = l4_field(proto);
  if (fo && tl - hl >= l4_min(proto)) put_field(at, i, hl + fo, res[2 * i + 1]);
}

template <class At>
void set_fields(uint64_t n, int mode, const uint16_t *res, const At &at) {
  const uint32_t f = mode_field(mode);
  auto one = [&](uint64_t i) {
    if (mode == YU_MODE_TX_DATAGRAM) {
      put_datagram_fields(at, i, res);
      return;
    }
    if (mode == YU_MODE_IPV4) {  // the field must lie inside the header
      const uint8_t *b0 = at(i, 0);
      if (!b0 || (uint32_t)(*b0 & 0xFu) * 4u < f + 2u) return;
    }
    put_field(at, i, f, res[i]);
  };
  constexpr uint64_t kParMin = 1u << 16;
  CopyPool &pool = CopyPool::get();
  const uint64_t parts = std::min<uint64_t>((uint64_t)pool.threads() + 1, n / kParMin);
  if (parts >= 2) {
    const uint64_t per = (n + parts - 1) / parts;
    if (pool.run((int)parts, [&](int k) {
          for (uint64_t i = (uint64_t)k * per; i < n && i < (uint64_t)(k + 1) * per; ++i) one(i);
        }))
      return;
  }
  for (uint64_t i = 0; i < n; ++i) one(i);
}

// Results into the caller's array, or a scratch one when it passes none
// (p stays null when that allocation fails: the call returns YU_ENOMEM, no
// exception crosses the C ABI).
struct ResultBuf {
  std::unique_ptr<uint16_t[]> tmp;
  uint16_t *p;
  ResultBuf(uint16_t *out, uint64_t n) : p(out) {  // n = results, not packets
    if (!p) {
      tmp.reset(new (std::nothrow) uint16_t[n ? n : 1]);
      p = tmp.get();
    }
  }
};

}  // namespace

extern "C" int yu_csum_fill_host_uniform(uint8_t *h_data, uint64_t stride, uint32_t len,
                                         uint64_t n, int mode, const uint16_t *h_initial_arr,
                                         uint16_t initial, const uint8_t *h_addrs,
                                         uint16_t *h_out, int device) {
  if (!tx_mode(mode)) return YU_EINVAL;  // EINVAL:fill-mode (bad mode too)
  if (n == 0) return YU_OK;
  ResultBuf r(h_out, n * YU_MODE_OUTPUTS(mode));
  if (!r.p) return YU_ENOMEM;
  int rc = yu_csum_batch_host_uniform(h_data, stride, len, n, mode, h_initial_arr, initial,
                                      h_addrs, r.p, device);
  if (rc) return rc;
  set_fields(n, mode, r.p, [&](uint64_t i, uint32_t k) -> uint8_t * {
    return k < len ? h_data + i * stride + k : nullptr;
  });
  return YU_OK;
}

extern "C" int yu_csum_fill_host_ragged(uint8_t *h_data, const uint64_t *h_offsets, uint64_t n,
                                        int mode, const uint16_t *h_initial_arr,
                                        uint16_t initial, const uint8_t *h_addrs,
                                        uint16_t *h_out, int device) {
  if (!tx_mode(mode)) return YU_EINVAL;  // EINVAL:fill-mode (bad mode too)
  if (n == 0) return YU_OK;
  ResultBuf r(h_out, n * YU_MODE_OUTPUTS(mode));
  if (!r.p) return YU_ENOMEM;
  int rc = yu_csum_batch_host_ragged(h_data, h_offsets, n, mode, h_initial_arr, initial, h_addrs,
                                     r.p, device);
  if (rc) return rc;
  set_fields(n, mode, r.p, [&](uint64_t i, uint32_t k) -> uint8_t * {
    return k < h_offsets[i + 1] - h_offsets[i] ? h_data + h_offsets[i] + k : nullptr;
  });
  return YU_OK;
}

extern "C" int yu_csum_fill_host_iov(const yu_iovec *iov, const uint64_t *first_iov, uint64_t n,
                                     int mode, const uint16_t *h_initial_arr, uint16_t initial,
                                     const uint8_t *h_addrs, uint16_t *h_out, int device) {
  if (!tx_mode(mode)) return YU_EINVAL;  // EINVAL:fill-mode (bad mode too)
  if (n == 0) return YU_OK;
  ResultBuf r(h_out, n * YU_MODE_OUTPUTS(mode));
  if (!r.p) return YU_ENOMEM;
  int rc = yu_csum_batch_host_iov(iov, first_iov, n, mode, h_initial_arr, initial, h_addrs, r.p,
                                  device);
  if (rc) return rc;
  // byte k of packet i: walk its views (the field may straddle two of them)
  set_fields(n, mode, r.p, [&](uint64_t i, uint32_t k) -> uint8_t * {
    uint64_t at = k;
    for (uint64_t v = first_iov[i]; v < first_iov[i + 1]; ++v) {
      if (at < iov[v].len) return (uint8_t *)iov[v].base + at;
      at -= iov[v].len;
    }
    return nullptr;
  });
  return YU_OK;
}
