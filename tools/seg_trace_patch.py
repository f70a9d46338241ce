"""Adds k_seg step tracing to a COPY of the kernel file (tools/side_build.sh <dir> <rev> tools/seg_trace_patch.py).

Debug side build only, read by tools/seg_trace.cpp: every 61st wave of k_seg records seven
shader-clock stamps per step (s_memtime, a read of the clock) and lane 0 stores them with
ordinary vector stores into a host-registered buffer set through yu_debug_set_trace().
The anchors are exact strings of the kernel file; the script fails if one is missing.
"""
import sys

p = sys.argv[1]
s=open(p).read()
def rep(old,new,count=1):
    global s
    assert s.count(old)==count, (s.count(old), old[:80])
    s=s.replace(old,new)
rep('''  uint32_t small_waves;  // k_seg: waves that work on small-packet batches (seg_waves)
  int mode;''','''  uint32_t small_waves;  // k_seg: waves that work on small-packet batches (seg_waves)
  uint64_t *trace;       // DEBUG (side build only): per-step timestamps of sampled waves
  int mode;''')
rep('''typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));''','''typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t tstamp(uint32_t dep) {
  uint64_t t;
  asm volatile("s_memtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "v"(dep));
  return t;
}''')
rep('''    const bool last = t * T + T >= cur.xe;  // wave-uniform
    SegChunk nn;''','''    const bool last = t * T + T >= cur.xe;  // wave-uniform
    const bool trw = A.trace && (wave % 61u) == 0u && trk < 64u;
    uint64_t trs[7];
    trs[0] = trw ? tstamp(0u) : 0u;
    auto trec = [&](uint32_t kind, uint32_t dep) __attribute__((always_inline)) {
      if (trw) {
        trs[6] = tstamp(dep);
        if (lane == 0u) {
          uint64_t *q = A.trace + ((wave / 61u) * 64u + trk) * 8u;
#pragma unroll
          for (int j = 0; j < 7; ++j) q[j] = trs[j];
          q[7] = kind | (t << 8);
        }
      }
      ++trk;
    };
    SegChunk nn;''')
rep('''    seg_fetch<U, NT != 0>(last ? nxt.b0 : cur.b0, last ? nxt.xe : cur.xe, last ? 0u : t + 1u, lane,
                          end, cn);
''','''    trs[1] = trw ? tstamp((uint32_t)nxt.b0) : 0u;
    seg_fetch<U, NT != 0>(last ? nxt.b0 : cur.b0, last ? nxt.xe : cur.xe, last ? 0u : t + 1u, lane,
                          end, cn);
    trs[2] = trw ? tstamp(c[0].x) : 0u;
    trs[3] = trw ? tstamp(c[U - 1].w) : 0u;
''')
rep('''    bool here = false;
#pragma unroll''','''    trs[4] = trw ? tstamp(carry_l) : 0u;
    bool here = false;
#pragma unroll''')
rep('''#pragma unroll
    for (int i = 0; i < NP; ++i)
      if (!(RX && i == 1) && pt[i].x - tb == T) pt[i].p = carry_l;''','''    trs[5] = trw ? tstamp(pt[0].p ^ pt[NP - 1].p) : 0u;
#pragma unroll
    for (int i = 0; i < NP; ++i)
      if (!(RX && i == 1) && pt[i].x - tb == T) pt[i].p = carry_l;''')
rep('''    if (!last) {
      ++t;
      return false;
    }
    // end sums: the next lane's start (ragged), else this lane's end point''','''    if (!last) {
      trec(0u, pt[0].p);
      ++t;
      return false;
    }
    // end sums: the next lane's start (ragged), else this lane's end point''')
rep('''    if ((ch + nwave) * CH >= A.n) return true;
    cur = nxt;''','''    trec(1u, pt[NP - 1].p ^ (uint32_t)cur.oy);
    if ((ch + nwave) * CH >= A.n) return true;
    cur = nxt;''')
rep('''  uint64_t t = 0;
  // One tile: issue the loads of the next item into cn, then sum c.''','''  uint64_t t = 0;
  uint32_t trk = 0;
  // One tile: issue the loads of the next item into cn, then sum c.''')
rep('''  a.small_waves = (uint32_t)cu_count(dev) * 4u * (uint32_t)seg_small_blocks();
''','''  a.small_waves = (uint32_t)cu_count(dev) * 4u * (uint32_t)seg_small_blocks();
  a.trace = g_debug_trace;
''')
rep('''int launch(const Variant &v, const BatchArgs &A, hipStream_t stream) {''','''uint64_t *g_debug_trace = nullptr;

int launch(const Variant &v, const BatchArgs &A, hipStream_t stream) {''')
rep('''extern "C" {

int yu_csum_batch_uniform(''','''extern "C" {

__attribute__((visibility("default"))) void yu_debug_set_trace(uint64_t *p) { g_debug_trace = p; }

int yu_csum_batch_uniform(''')
open(p,'w').write(s)
