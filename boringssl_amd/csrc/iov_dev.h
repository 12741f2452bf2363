// iov_dev.h -- device helpers shared by the bulk kernels (gcm.hip, chacha.hip):
// partial 16-byte loads / stores of record bytes and the in-place walk of
// iovec records (BatchDesc::iovecs).
#ifndef BSSL_AMD_IOV_DEV_H
#define BSSL_AMD_IOV_DEV_H

#include <hip/hip_runtime.h>

#include "internal.h"

namespace bssl_amd {
namespace {

// 16-byte block loads and stores at any address.  The HSA runtime runs the
// shader memory in unaligned mode (SH_MEM_CONFIG.alignment_mode), so
// global_load/store_dwordx4 take byte addresses; the 1-byte-aligned type lets
// the compiler emit them for records that are not 16-byte aligned (the same
// instruction an aligned block uses; an unaligned one costs its extra cache
// line in the TA, nothing on the VALU).
typedef uint32_t u32_any __attribute__((aligned(1)));

// Record buffers are device memory, and every helper below reaches them
// through global-address-space pointers (gptr): a pointer read from a chunk
// descriptor is otherwise a generic one, and a generic (flat_*) access counts
// on lgkmcnt as well as vmcnt, so each LDS wait after it -- the AES table
// lookups of the rounds -- would also wait for that HBM access.
#define BSSL_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ BSSL_GLOBAL T *gptr(T *p) {
  return (BSSL_GLOBAL T *)p;
}

// Integer min of two 64-bit lengths.  (HIP's min<uint64_t> in device code
// goes through double precision: two conversions and v_min_f64.)
__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

__device__ __forceinline__ uint4 load16_any(const uint8_t *p) {
  const BSSL_GLOBAL u32_any *ip = (const BSSL_GLOBAL u32_any *)p;
  return make_uint4(ip[0], ip[1], ip[2], ip[3]);
}

__device__ __forceinline__ void store16_any(uint8_t *p, uint4 v) {
  BSSL_GLOBAL u32_any *o = (BSSL_GLOBAL u32_any *)p;
  o[0] = v.x;
  o[1] = v.y;
  o[2] = v.z;
  o[3] = v.w;
}

// ---------------------------------------------------------------------------
// Record buffers.
// Bytes [p, p + n) (n <= 16), zero past n, with aligned dword loads: only
// dwords holding at least one of the bytes are read (they lie in the same
// pages as those bytes), then funnel-shifted.  (Byte loads cost one memory
// request per byte.)
__device__ __forceinline__ uint4 load_partial(const uint8_t *p, uint32_t n) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const BSSL_GLOBAL uint32_t *base = (const BSSL_GLOBAL uint32_t *)(a & ~uintptr_t(3));
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t nd = n ? (sh + n + 3) / 4 : 0u;  // dwords touched
  uint32_t d[5];
#pragma unroll
  for (int k = 0; k < 5; k++) d[k] = (uint32_t)k < nd ? base[k] : 0u;
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t v = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
    const uint32_t lo = 4u * i;
    w[i] = v & ((n >= lo + 4) ? 0xffffffffu : (n <= lo) ? 0u : ((1u << (8 * (n - lo))) - 1u));
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Bytes [0, n) of v to p: one 16-byte store for a whole aligned block,
// dword (+ short / byte) stores when p is 4-byte aligned, else dword stores
// at the byte address and the last 1-3 bytes.  (Each narrow store is a
// memory request of its own; a record's tag and tail otherwise cost up to 31
// of them.)
__device__ __forceinline__ void store_partial(uint8_t *p, uint4 v, uint32_t n) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  if (n >= 16 && (a & 15) == 0) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    *(BSSL_GLOBAL v4u *)p = v4u{v.x, v.y, v.z, v.w};
  } else if ((a & 3) == 0) {
    BSSL_GLOBAL uint32_t *pw = (BSSL_GLOBAL uint32_t *)p;
    uint32_t last = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if (4u * i + 4 <= n) pw[i] = w[i];
      if (n / 4 == (uint32_t)i) last = w[i];
    }
    const uint32_t r = n & 3;
    if (r) {
      BSSL_GLOBAL uint8_t *q = gptr(p) + (n & ~3u);
      if (r & 2) *(BSSL_GLOBAL uint16_t *)q = (uint16_t)last;
      if (r & 1) q[r & 2] = (uint8_t)(last >> (8 * (r & 2)));
    }
  } else {
    // Unaligned: whole dwords at byte addresses (unaligned mode, as
    // store16_any), then the last 1-3 bytes.
    BSSL_GLOBAL u32_any *pw = (BSSL_GLOBAL u32_any *)p;
    uint32_t last = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if (4u * i + 4 <= n) pw[i] = w[i];
      if (n / 4 == (uint32_t)i) last = w[i];
    }
    BSSL_GLOBAL uint8_t *q = gptr(p) + (n & ~3u);
    for (uint32_t i = 0; i < (n & 3); i++) q[i] = (uint8_t)(last >> (8 * i));
  }
}

__device__ __forceinline__ uint4 mask_block(uint4 v, uint32_t n) {
  if (n >= 16) return v;
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t lo = 4 * i;
    const uint32_t m = (n >= lo + 4) ? 0xffffffffu : (n <= lo) ? 0u : ((1u << (8 * (n - lo))) - 1u);
    w[i] &= m;
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// ---------------------------------------------------------------------------
// iovec records walked in place (BatchDesc::iovecs; reference
// EVP_AEAD_CTX_sealv / _openv_detached, aead.cc.inc:316-361, 531-584, whose
// AEADs walk the chunks with ForEachBlockRange, cipher/internal.h:283-411).
// A lane keeps a cursor on the chunk holding its current stream position:
// chunk c covers stream bytes [cs, ce) of the record.
struct IovCur {
  uint64_t c, cs, ce;
  const uint8_t *in;
  uint8_t *out;
};

// Chunk descriptors come through a source D: d(c) is chunk c of the batch.
// IovDescG reads them from the batch's array in device memory; a kernel may
// pass a source that serves a record's first chunks from LDS (gcm.hip).
struct IovDescG {
  const IovecDev *v;
  __device__ __forceinline__ IovecDev operator()(uint64_t c) const { return v[c]; }
};

template <class D>
__device__ __forceinline__ void iov_at_d(IovCur &k, const D &d, uint64_t c, uint64_t cs) {
  const IovecDev v = d(c);
  k.c = c;
  k.cs = cs;
  k.ce = cs + v.len;
  k.in = v.in;
  k.out = v.out;
}

// Advance to the chunk holding stream byte p (positions only grow).
template <class D>
__device__ __forceinline__ void iov_seek_d(IovCur &k, const D &d, uint64_t p, uint64_t c_end) {
  while (p >= k.ce && k.c + 1 < c_end) iov_at_d(k, d, k.c + 1, k.ce);
}

__device__ __forceinline__ void iov_at(IovCur &k, const BatchDesc &b, uint64_t c, uint64_t cs) {
  iov_at_d(k, IovDescG{b.iovecs}, c, cs);
}

__device__ __forceinline__ void iov_seek(IovCur &k, const BatchDesc &b, uint64_t p,
                                         uint64_t c_end) {
  iov_seek_d(k, IovDescG{b.iovecs}, p, c_end);
}

// The cursor of chunk c (stream start cs), advanced to the chunk holding p.
__device__ __forceinline__ IovCur iov_cur_at(const BatchDesc &b, uint64_t c, uint64_t cs,
                                             uint64_t p, uint64_t c_end) {
  IovCur k;
  iov_at(k, b, c, cs);
  iov_seek(k, b, p, c_end);
  return k;
}

template <class D>
__device__ __forceinline__ IovCur iov_cur_at_d(const D &d, uint64_t c, uint64_t cs, uint64_t p,
                                               uint64_t c_end) {
  IovCur k;
  iov_at_d(k, d, c, cs);
  iov_seek_d(k, d, p, c_end);
  return k;
}

template <class D>
__device__ __forceinline__ uint64_t iov_len_at_d(const D &d, uint64_t c, uint64_t c_end) {
  return c < c_end ? d(c).len : 0;
}

// Length of chunk c of a record whose chunks end at c_end (0 past the end).
__device__ __forceinline__ uint64_t iov_len_at(const BatchDesc &b, uint64_t c, uint64_t c_end) {
  return c < c_end ? b.iovecs[c].len : 0;
}

// Bytes [a, a + 16) of the 32 bytes A || B (a = 0..16).
__device__ __forceinline__ uint4 bytes_at(uint4 A, uint4 B, uint32_t a) {
  const uint32_t w[9] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w, 0u};
  const uint32_t wq = a >> 2, r = a & 3;
  uint32_t t[5];
#pragma unroll
  for (int i = 0; i < 5; i++)
    t[i] = wq == 0 ? w[i] : wq == 1 ? w[i + 1] : wq == 2 ? w[i + 2] : wq == 3 ? w[i + 3] : w[i + 4];
  return make_uint4(__builtin_amdgcn_alignbyte(t[1], t[0], r),
                    __builtin_amdgcn_alignbyte(t[2], t[1], r),
                    __builtin_amdgcn_alignbyte(t[3], t[2], r),
                    __builtin_amdgcn_alignbyte(t[4], t[3], r));
}

// Bytes [p, p + n) (n <= 16, zero past n) of a block that ends in chunk k.c
// or the next chunk (the usual straddle: at most one boundary): one partial
// load per piece, joined by a byte shift.  Returns false (nothing loaded)
// when more chunks are involved.
template <class D>
__device__ __forceinline__ bool iov_load2_d(const D &d, const IovCur &k, uint64_t p, uint32_t n,
                                            uint64_t c_end, uint4 &v) {
  const uint32_t n1 = (uint32_t)umin64(n, k.ce - p);
  uint4 v2 = make_uint4(0, 0, 0, 0);
  if (n1 < n) {
    if (k.c + 1 >= c_end) return false;
    const IovecDev nx = d(k.c + 1);
    if (nx.len < n - n1) return false;
    v2 = load_partial(nx.in, n - n1);
  }
  const uint4 v1 = load_partial(k.in + (p - k.cs), n1);
  const uint4 s2 = bytes_at(make_uint4(0, 0, 0, 0), v2, 16 - n1);  // v2 << 8 n1
  v = make_uint4(v1.x | s2.x, v1.y | s2.y, v1.z | s2.z, v1.w | s2.w);
  return true;
}

template <class D>
__device__ __forceinline__ bool iov_store2_d(const D &d, const IovCur &k, uint64_t p, uint4 y,
                                             uint32_t n, uint64_t c_end) {
  const uint32_t n1 = (uint32_t)umin64(n, k.ce - p);
  IovecDev nx = {nullptr, nullptr, 0};
  if (n1 < n) {
    if (k.c + 1 >= c_end) return false;
    nx = d(k.c + 1);
    if (nx.len < n - n1) return false;
  }
  store_partial(k.out + (p - k.cs), y, n1);
  if (n1 < n) store_partial(nx.out, bytes_at(y, make_uint4(0, 0, 0, 0), n1), n - n1);
  return true;
}

// Bytes [p, p + n) of the record's stream (n <= 16, zero past n), byte by
// byte across chunk boundaries (blocks over three or more chunks).
template <class D>
__device__ __forceinline__ uint4 iov_gather_d(const D &d, IovCur k, uint64_t p, uint32_t n,
                                              uint64_t c_end) {
  uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
  for (uint32_t i = 0; i < n; i++) {
    iov_seek_d(k, d, p + i, c_end);
    const uint32_t v = (uint32_t)gptr(k.in)[p + i - k.cs] << (8 * (i & 3));
    const uint32_t wi = i >> 2;
    w0 |= wi == 0 ? v : 0u;
    w1 |= wi == 1 ? v : 0u;
    w2 |= wi == 2 ? v : 0u;
    w3 |= wi == 3 ? v : 0u;
  }
  return make_uint4(w0, w1, w2, w3);
}

template <class D>
__device__ __forceinline__ void iov_scatter_d(const D &d, IovCur k, uint64_t p, uint4 y,
                                              uint32_t n, uint64_t c_end) {
  const uint32_t w[4] = {y.x, y.y, y.z, y.w};
  for (uint32_t i = 0; i < n; i++) {
    iov_seek_d(k, d, p + i, c_end);
    const uint32_t wi = i >> 2;
    const uint32_t v = wi == 0 ? w[0] : wi == 1 ? w[1] : wi == 2 ? w[2] : w[3];
    gptr(k.out)[p + i - k.cs] = (uint8_t)(v >> (8 * (i & 3)));
  }
}

__device__ __forceinline__ bool iov_load2(const BatchDesc &b, const IovCur &k, uint64_t p,
                                          uint32_t n, uint64_t c_end, uint4 &v) {
  return iov_load2_d(IovDescG{b.iovecs}, k, p, n, c_end, v);
}

__device__ __forceinline__ bool iov_store2(const BatchDesc &b, const IovCur &k, uint64_t p,
                                           uint4 y, uint32_t n, uint64_t c_end) {
  return iov_store2_d(IovDescG{b.iovecs}, k, p, y, n, c_end);
}

__device__ __forceinline__ uint4 iov_gather(const BatchDesc &b, IovCur k, uint64_t p, uint32_t n,
                                            uint64_t c_end) {
  return iov_gather_d(IovDescG{b.iovecs}, k, p, n, c_end);
}

__device__ __forceinline__ void iov_scatter(const BatchDesc &b, IovCur k, uint64_t p, uint4 y,
                                            uint32_t n, uint64_t c_end) {
  iov_scatter_d(IovDescG{b.iovecs}, k, p, y, n, c_end);
}

// Chunk descriptors of an iovec record from an LDS slot (gcm.hip, chacha.hip):
// the record's chunk range [c0, c_end) at +0 / +8 and its chunks c0 .. c0+KC-1
// at +16 + 32 i (out, in, len), copied by the record's lanes when the record
// starts; later chunks come from the batch's array.  The record's walks then
// issue no global load before the block load itself: a chunk-table load
// issued after the previous blocks' stores waits for all of them (vmcnt counts
// loads and stores in issue order), an LDS read does not.
template <uint32_t KC>
constexpr uint32_t kIovSlotBytes = 16u + 32u * KC;

template <uint32_t KC>
struct IovDescL {
  const uint8_t *ls;  // the record's slot
  uint64_t c0;
  const IovecDev *g;
  __device__ __forceinline__ IovecDev operator()(uint64_t c) const {
    if (c - c0 < KC) {
      const uint8_t *d = ls + 16u + (uint32_t)(c - c0) * 32u;
      const uint4 w = *reinterpret_cast<const uint4 *>(d);
      IovecDev v;
      v.out = reinterpret_cast<uint8_t *>(((uint64_t)w.y << 32) | w.x);
      v.in = reinterpret_cast<const uint8_t *>(((uint64_t)w.w << 32) | w.z);
      v.len = *reinterpret_cast<const uint64_t *>(d + 16);
      return v;
    }
    // (Wait for the fallback's load here: otherwise the join with the LDS
    // path leaves the descriptor pending on vmcnt, and the walk waits for
    // every outstanding load and store even when it read LDS.)
    uint64_t o = reinterpret_cast<uint64_t>(g[c].out), i = reinterpret_cast<uint64_t>(g[c].in),
             len = g[c].len;
    asm volatile("" : "+v"(o), "+v"(i), "+v"(len));
    IovecDev v;
    v.out = reinterpret_cast<uint8_t *>(o);
    v.in = reinterpret_cast<const uint8_t *>(i);
    v.len = len;
    return v;
  }
};

// Fill the slot of live record rec (first chunk c0) from its L lanes (lane q
// of the record copies chunks c0 + q, c0 + q + L, ...).  The caller then runs
// iov_slot_sync() with the whole wave.
template <uint32_t KC, int L>
__device__ __forceinline__ void iov_slot_fill(uint8_t *ls, const BatchDesc &b, uint64_t rec,
                                              uint64_t c0, int q) {
  const uint64_t ce = b.iovec_start[rec + 1];
  if (q == 0)
    *reinterpret_cast<uint4 *>(ls) =
        make_uint4((uint32_t)c0, (uint32_t)(c0 >> 32), (uint32_t)ce, (uint32_t)(ce >> 32));
#pragma unroll
  for (uint32_t i = (uint32_t)q; i < KC; i += (uint32_t)L) {
    if (c0 + i < ce) {
      const IovecDev v = b.iovecs[c0 + i];
      const uint64_t o = reinterpret_cast<uint64_t>(v.out), n = reinterpret_cast<uint64_t>(v.in);
      *reinterpret_cast<uint4 *>(ls + 16 + 32 * i) =
          make_uint4((uint32_t)o, (uint32_t)(o >> 32), (uint32_t)n, (uint32_t)(n >> 32));
      *reinterpret_cast<uint64_t *>(ls + 16 + 32 * i + 16) = v.len;
    }
  }
}

// (A slot is written and read by the lanes of one wave, whose LDS accesses
// complete in issue order; the fences keep the compiler from moving the
// slot's reads above the fill.)
__device__ __forceinline__ void iov_slot_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The descriptor source of a filled slot and the record's chunk end.
template <uint32_t KC>
__device__ __forceinline__ IovDescL<KC> iov_slot_src(const uint8_t *ls, const BatchDesc &b,
                                                     uint64_t &c_end) {
  const uint4 h = *reinterpret_cast<const uint4 *>(ls);
  c_end = ((uint64_t)h.w << 32) | h.z;
  return IovDescL<KC>{ls, ((uint64_t)h.y << 32) | h.x, b.iovecs};
}

// Bytes [pos, pos + n) of the concatenation of chunks v[c0 .. c1) (AD of an
// iovec record; n <= 16, zero past n).  Walks from c0: the AD is short.
__device__ __forceinline__ uint4 ivec_load16(const IvecDev *v, uint64_t c0, uint64_t c1,
                                             uint64_t pos, uint32_t n) {
  if (c0 < c1) {  // inside the first chunk (TLS: one chunk of 13 bytes): one partial load
    const IvecDev f = v[c0];
    if (pos + n <= f.len) return load_partial(f.in + pos, n);
  }
  uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
  uint64_t c = c0, cs = 0;
  for (uint32_t i = 0; i < n; i++) {
    while (c < c1 && pos + i >= cs + v[c].len) {
      cs += v[c].len;
      c++;
    }
    const uint32_t x = (uint32_t)v[c].in[pos + i - cs] << (8 * (i & 3));
    const uint32_t wi = i >> 2;
    w0 |= wi == 0 ? x : 0u;
    w1 |= wi == 1 ? x : 0u;
    w2 |= wi == 2 ? x : 0u;
    w3 |= wi == 3 ? x : 0u;
  }
  return make_uint4(w0, w1, w2, w3);
}

// A lane's walk over one iovec record at a fixed stride: the lane reads (or
// writes) 16-byte blocks at stream positions p, p + stride, ...  Between chunk
// boundaries only a running pointer moves (`left` = bytes of the chunk from
// the next block on; >= 16: the next block is one dwordx4 at `ptr`); a chunk
// boundary, a partial block or the first block take the cursor path (seek,
// one or two partial accesses, the byte walk over three or more chunks).
struct IovWalk {
  uint64_t c, cs;  // chunk index and its stream start
  uint8_t *ptr;
  int64_t left;
};

__device__ __forceinline__ void iov_walk_init(IovWalk &w, const BatchDesc &b, uint64_t rec) {
  w.c = b.iovec_start[rec];
  w.cs = 0;
  w.ptr = nullptr;
  w.left = -1;
}

// Bytes [p, p + n) of the record (n = 1..16, zero past n).
__device__ __forceinline__ uint4 iov_walk_load(IovWalk &w, const BatchDesc &b, uint64_t rec,
                                               uint64_t p, uint32_t n, uint32_t stride) {
  uint4 v;
  if (n == 16 && w.left >= 16) {
    v = load16_any(w.ptr);
    w.ptr += stride;
    w.left -= stride;
    return v;
  }
  const uint64_t c_end = b.iovec_start[rec + 1];
  IovCur k;
  iov_at(k, b, w.c, w.cs);
  iov_seek(k, b, p, c_end);
  if (n == 16 && p + 16 <= k.ce)
    v = load16_any(k.in + (p - k.cs));
  else if (!iov_load2(b, k, p, n, c_end, v))
    v = iov_gather(b, k, p, n, c_end);
  w.c = k.c;
  w.cs = k.cs;
  w.ptr = const_cast<uint8_t *>(k.in) + (p - k.cs) + stride;
  w.left = (int64_t)(k.ce - p) - (int64_t)stride;
  return v;
}

// Bytes [0, n) of y to stream positions [p, p + n).
__device__ __forceinline__ void iov_walk_store(IovWalk &w, const BatchDesc &b, uint64_t rec,
                                               uint64_t p, uint4 y, uint32_t n, uint32_t stride) {
  if (n == 16 && w.left >= 16) {
    store16_any(w.ptr, y);
    w.ptr += stride;
    w.left -= stride;
    return;
  }
  const uint64_t c_end = b.iovec_start[rec + 1];
  IovCur k;
  iov_at(k, b, w.c, w.cs);
  iov_seek(k, b, p, c_end);
  if (n == 16 && p + 16 <= k.ce)
    store16_any(k.out + (p - k.cs), y);
  else if (!iov_store2(b, k, p, y, n, c_end))
    iov_scatter(b, k, p, y, n, c_end);
  w.c = k.c;
  w.cs = k.cs;
  w.ptr = k.out + (p - k.cs) + stride;
  w.left = (int64_t)(k.ce - p) - (int64_t)stride;
}

// Zeroes an iovec record's output chunks (clear_iovec, aead.cc.inc:310-333),
// lane q of L lanes writing bytes q, q + L, ...
__device__ __forceinline__ void iov_clear(const BatchDesc &b, uint64_t rec, int q, int L) {
  for (uint64_t c = b.iovec_start[rec]; c < b.iovec_start[rec + 1]; c++) {
    const IovecDev v = b.iovecs[c];
    for (uint64_t i = q; i < v.len; i += L) v.out[i] = 0;
  }
}

}  // namespace
}  // namespace bssl_amd

#endif
