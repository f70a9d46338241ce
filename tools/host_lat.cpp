// host_lat.cpp — measurement tool (not product): where the per-call time of a
// small host-memory batch goes (HIP API calls vs launch + sync vs the call).
//
// build: hipcc -O2 --offload-arch=gfx950 -I include tools/host_lat.cpp -o tools/host_lat -L yustack_amd -lyucsum -Wl,-rpath,'$ORIGIN/../yustack_amd'
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <vector>

#include "yucsum.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

__global__ void empty_kernel(int *p) {
  if (p && threadIdx.x == 1000) p[0] = 1;
}

// Completion flag in pinned host memory, written after everything before it
// on the stream (system-scope release).
__global__ void flag_kernel(volatile unsigned *flag, unsigned v) {
  __threadfence_system();
  *flag = v;
  __threadfence_system();
}

// The flag written by the kernel itself: the last of its blocks to finish
// (device-scope counter, reset by that block) stores it, so no second launch.
__global__ void empty_then_flag(unsigned *ctr, volatile unsigned *flag, unsigned v) {
  __shared__ bool last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(ctr, 1u) == gridDim.x - 1u;
  }
  __syncthreads();
  if (last && threadIdx.x == 0) {
    *ctr = 0u;
    __threadfence_system();
    *flag = v;
  }
}

template <class F>
static double per_call_us(int reps, F &&f) {
  for (int i = 0; i < 20; ++i) f();
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps; ++i) f();
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}

int main() {
  const int reps = 2000;
  const uint32_t L = 1500;
  const uint64_t n = 64;
  uint8_t *pinned, *addrs;
  uint16_t *out;
  CK(hipHostMalloc((void **)&pinned, n * L, 0));
  CK(hipHostMalloc((void **)&addrs, n * 8, 0));
  CK(hipHostMalloc((void **)&out, n * 2, 0));
  for (uint64_t i = 0; i < n * L; ++i) pinned[i] = (uint8_t)(i * 131);
  for (uint64_t i = 0; i < n; ++i) pinned[i * L + 12] = 0x50;
  std::vector<uint8_t> pageable(pinned, pinned + n * L);
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));

  hipPointerAttribute_t a;
  printf("hipPointerGetAttributes (pinned):  %6.2f us\n",
         per_call_us(reps, [&] { (void)hipPointerGetAttributes(&a, pinned + 17); }));
  printf("hipPointerGetAttributes (pageable):%6.2f us\n", per_call_us(reps, [&] {
           if (hipPointerGetAttributes(&a, pageable.data()) != hipSuccess) (void)hipGetLastError();
         }));
  void *d;
  printf("hipHostGetDevicePointer:           %6.2f us\n",
         per_call_us(reps, [&] { (void)hipHostGetDevicePointer(&d, pinned, 0); }));
  printf("hipGetDevice + hipSetDevice:       %6.2f us\n", per_call_us(reps, [&] {
           int dev;
           (void)hipGetDevice(&dev);
           (void)hipSetDevice(dev);
         }));
  printf("empty kernel launch only:          %6.2f us\n",
         per_call_us(reps, [&] { empty_kernel<<<1, 64, 0, st>>>(nullptr); }));
  CK(hipStreamSynchronize(st));
  printf("empty kernel launch + sync:        %6.2f us\n", per_call_us(reps, [&] {
           empty_kernel<<<1, 64, 0, st>>>(nullptr);
           (void)hipStreamSynchronize(st);
         }));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  printf("empty launch + event + query spin: %6.2f us\n", per_call_us(reps, [&] {
           empty_kernel<<<1, 64, 0, st>>>(nullptr);
           (void)hipEventRecord(ev, st);
           while (hipEventQuery(ev) == hipErrorNotReady) {
           }
         }));
  printf("empty launch + stream query spin:  %6.2f us\n", per_call_us(reps, [&] {
           empty_kernel<<<1, 64, 0, st>>>(nullptr);
           while (hipStreamQuery(st) == hipErrorNotReady) {
           }
         }));
  unsigned *flag;
  CK(hipHostMalloc((void **)&flag, 64, 0));
  unsigned seq = 0;
  printf("empty launch + flag kernel + poll: %6.2f us\n", per_call_us(reps, [&] {
           ++seq;
           empty_kernel<<<1, 64, 0, st>>>(nullptr);
           flag_kernel<<<1, 1, 0, st>>>(flag, seq);
           while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
           }
         }));
  CK(hipStreamSynchronize(st));
  printf("empty launch + hipStreamWriteValue32 + poll: %6.2f us\n", per_call_us(reps, [&] {
           ++seq;
           empty_kernel<<<1, 64, 0, st>>>(nullptr);
           (void)hipStreamWriteValue32(st, flag, seq, 0);
           while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
           }
         }));
  CK(hipStreamSynchronize(st));
  unsigned *ctr;
  CK(hipMalloc((void **)&ctr, 4));
  CK(hipMemset(ctr, 0, 4));
  for (int blocks : {1, 64, 1024}) {
    printf("kernel (%4d blocks) storing the flag itself + poll: %6.2f us\n", blocks, per_call_us(reps, [&] {
             ++seq;
             empty_then_flag<<<blocks, 256, 0, st>>>(ctr, flag, seq);
             while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
             }
           }));
    CK(hipStreamSynchronize(st));
  }
  printf("batch kernel + flag kernel + poll: %6.2f us\n", per_call_us(reps, [&] {
           ++seq;
           (void)yu_csum_batch_uniform(pinned, L, L, n, YU_MODE_TCP, nullptr, 0, addrs, out, st);
           flag_kernel<<<1, 1, 0, st>>>(flag, seq);
           while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
           }
         }));
  CK(hipStreamSynchronize(st));
  printf("batch kernel on pinned, + sync:    %6.2f us\n", per_call_us(reps, [&] {
           (void)yu_csum_batch_uniform(pinned, L, L, n, YU_MODE_TCP, nullptr, 0, addrs, out, st);
           (void)hipStreamSynchronize(st);
         }));
  printf("yu_csum_batch_host_uniform pinned: %6.2f us\n", per_call_us(reps, [&] {
           (void)yu_csum_batch_host_uniform(pinned, L, L, n, YU_MODE_TCP, nullptr, 0, addrs, out, 0);
         }));
  printf("yu_csum_batch_host_uniform pageable:%5.2f us\n", per_call_us(reps, [&] {
           (void)yu_csum_batch_host_uniform(pageable.data(), L, L, n, YU_MODE_TCP, nullptr, 0, addrs,
                                            out, 0);
         }));
  return 0;
}
