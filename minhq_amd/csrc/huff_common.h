// huff_common.h -- device helpers shared by the gfx950 codec kernels.
//
// Tiles: every kernel walks tiles of consecutive literals, one tile per wave
// at a time.  A tile's offsets come in as coalesced u64 loads (kept in
// registers, lane + 64k), its bytes are staged into the wave's LDS slice with
// aligned 16-B loads, and outputs leave the LDS slice as aligned 16-B stores.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mhq {
namespace dev {

constexpr int kWave = 64;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#ifdef MHQ_DBG_CRUMBS
// Diagnostic build (-DMHQ_DBG_CRUMBS): before each global access of the read
// path a lane records (site, address) in pinned host memory, which the host
// can still read after a GPU memory fault has taken the context down
// (mhq_dbg_crumbs_dump, read_strings.hip).  Null: not recording.
__device__ unsigned long long *g_crumbs;
__device__ __forceinline__ void crumb(uint32_t site, const void *p) {
  unsigned long long *c = g_crumbs;
  if (!c) return;
  c += 2ull * ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x);
  __hip_atomic_store(c + 1, (unsigned long long)(uintptr_t)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(c, (unsigned long long)site, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
#define CRUMB(site, p) ::mhq::dev::crumb((site), (const void *)(p))
#else
#define CRUMB(site, p) ((void)0)
#endif

// Orders this wave's LDS accesses (they retire in order per wave; this keeps
// the compiler from moving them across a phase boundary).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t popc64(uint64_t m) { return (uint32_t)__popcll(m); }

// Inclusive sum over lanes 0..lane of a full wave, in DPP moves (VALU only,
// no LDS round trips): prefix sums inside rows of 16 by row_shr 1/2/4/8, then
// row 15's total into rows 1 and 3 (row_bcast:15) and lane 31's into rows 2
// and 3 (row_bcast:31).  Every lane must be active.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}

template <int kTileLits>
struct TileOffsets {
  static constexpr int kPer = (kTileLits + 1 + kWave - 1) / kWave;
  uint64_t io[kPer];  // in_off[s + lane + 64k]
  uint64_t oo[kPer];  // out_off[s + lane + 64k] (unused by encode_len)

  __device__ __forceinline__ void load(const uint64_t *__restrict__ in_off, const uint64_t *__restrict__ out_off,
                                       uint64_t s, uint32_t cnt, int lane) {
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const uint32_t j = (uint32_t)lane + (uint32_t)k * kWave;
      io[k] = j <= cnt ? __builtin_nontemporal_load(in_off + s + j) : 0;
      oo[k] = (out_off && j <= cnt) ? __builtin_nontemporal_load(out_off + s + j) : 0;
    }
  }

  // Literals [cur, end] fit when their input span (from the 16-B aligned start)
  // is <= in_lim and their output span <= out_lim.  Returns end (>= cur; == cur
  // means literal `cur` alone does not fit).
  __device__ __forceinline__ uint32_t fit(uint32_t cur, uint32_t cnt, uint64_t in_lo, uint64_t in_lim,
                                          uint64_t out_lo, uint64_t out_lim, int lane) const {
    uint32_t n = 0;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const uint32_t j = (uint32_t)lane + (uint32_t)k * kWave;
      const bool ok = j > cur && j <= cnt && (io[k] - in_lo) <= in_lim && (oo[k] - out_lo) <= out_lim;
      n += popc64(__ballot(ok));
    }
    return cur + n;
  }
};

// First index i in [0, m) with key(i) >= target, or m.
template <class K>
__device__ __forceinline__ uint32_t lower_bound(K key, uint32_t m, uint32_t target) {
  uint32_t lo = 0, hi = m;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (key(mid) < target) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Byte-balanced split of literals [0, m) (input byte starts key(i)) into 64
// contiguous runs, one per lane.
template <class K>
__device__ __forceinline__ void lane_run(K key, uint32_t m, int lane, uint32_t &first, uint32_t &last) {
  const uint32_t b0 = key(0);
  const uint32_t total = key(m) - b0;
  const uint32_t t0 = b0 + (uint32_t)(((uint64_t)total * (uint32_t)lane) >> 6);
  const uint32_t t1 = b0 + (uint32_t)(((uint64_t)total * (uint32_t)(lane + 1)) >> 6);
  first = lane == 0 ? 0u : lower_bound(key, m, t0);
  last = lane == kWave - 1 ? m : lower_bound(key, m, t1);
}

// Ascending bitonic sort of 128 keys held two per lane: element i lives in
// lane i & 63, slot i >> 6 (v0: i = lane, v1: i = lane + 64).
__device__ __forceinline__ void sort128(uint32_t &v0, uint32_t &v1, int lane) {
#pragma unroll
  for (int k = 2; k <= 128; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j == 64) {
        const uint32_t lo = v0 < v1 ? v0 : v1, hi = v0 < v1 ? v1 : v0;
        v0 = lo;
        v1 = hi;
      } else {
        const uint32_t o0 = __shfl_xor(v0, j), o1 = __shfl_xor(v1, j);
        const bool lower = (lane & j) == 0;          // i < partner
        const bool asc0 = (lane & k) == 0;            // element lane
        const bool asc1 = ((lane + 64) & k) == 0;     // element lane + 64
        const bool min0 = lower == asc0, min1 = lower == asc1;
        v0 = min0 ? (v0 < o0 ? v0 : o0) : (v0 < o0 ? o0 : v0);
        v1 = min1 ? (v1 < o1 ? v1 : o1) : (v1 < o1 ? o1 : v1);
      }
    }
  }
}

// Copies global bytes [a, a+nbytes) (a 16-B aligned) into LDS words; kSwap
// byte-swaps every word (MSB-first bit streams); kReverse stores logical word
// w at index nwords-1-w so that {w+1, w} is one little-endian u64 pair.
template <bool kSwap, bool kReverse>
__device__ __forceinline__ void stage_in(uint32_t *lds, uint32_t nwords, const uint8_t *a, uint32_t nbytes,
                                         int lane) {
  const uint32_t chunks = (nbytes + 15u) >> 4;
  const u32x4 *src = (const u32x4 *)a;
  for (uint32_t c = lane; c < chunks; c += kWave) {
    u32x4 v = __builtin_nontemporal_load(src + c);  // an aligned chunk holding a valid byte never crosses a page
    if (kSwap) {
      v.x = __builtin_bswap32(v.x);
      v.y = __builtin_bswap32(v.y);
      v.z = __builtin_bswap32(v.z);
      v.w = __builtin_bswap32(v.w);
    }
    if (kReverse) {
      *(u32x4 *)(lds + nwords - 4u - 4u * c) = v.wzyx;
    } else {
      *(u32x4 *)(lds + 4u * c) = v;
    }
  }
}

__device__ __forceinline__ void zero_lds(uint32_t *lds, uint32_t nbytes, int lane) {
  const uint32_t chunks = (nbytes + 15u) >> 4;
  for (uint32_t c = lane; c < chunks; c += kWave) *(u32x4 *)(lds + 4u * c) = u32x4{0u, 0u, 0u, 0u};
}

// Writes LDS bytes [lo, hi) to global o_al + [lo, hi), o_al 16-B aligned.
// Whole 16-B chunks go out as one aligned store each; the bytes of the (at
// most two) partial chunks at the ends, at most 15 each, are written one per
// thread by threads 0-15 (head) and 16-31 (tail), all in one pass, so
// neighbours are untouched.  `lane` / `nthreads` (>= 32): this thread's index
// among the threads sharing the copy.
__device__ __forceinline__ void store_out(uint8_t *o_al, const uint8_t *lds, uint32_t lo, uint32_t hi, int lane,
                                          uint32_t nthreads = kWave) {
  if (hi <= lo) return;
  CRUMB(40, o_al + hi - 1);
  const uint32_t f0 = (lo + 15u) >> 4, f1 = hi >> 4;  // whole chunks [f0, f1)
  for (uint32_t c = f0 + lane; c < f1; c += nthreads)
    __builtin_nontemporal_store(*(const u32x4 *)(lds + (c << 4)), (u32x4 *)(o_al + (c << 4)));
  const uint32_t head_end = min(hi, f0 << 4), tail_start = max(head_end, f1 << 4);
  const uint32_t x = lane < 16 ? lo + (uint32_t)lane : tail_start + (uint32_t)lane - 16u;
  if (lane < 32 && x < (lane < 16 ? head_end : hi)) o_al[x] = lds[x];
}

// store_out for a slice of at most kMax wave-wide rounds of whole chunks
// (kMax * 64 * 16 bytes): every LDS read is issued before the first global
// store, so the copy waits for one LDS round trip, not one per round (the
// loop form waits after each ds_read_b128; under the probe loops' LDS load a
// round trip is hundreds of cycles).  Reads past the last whole chunk re-read
// it (no branch around a read); only the stores are predicated.
template <int kMax>
__device__ __forceinline__ void store_out_batched(uint8_t *o_al, const uint8_t *lds, uint32_t lo, uint32_t hi,
                                                  int lane) {
  if (hi <= lo) return;
  CRUMB(40, o_al + hi - 1);
  const uint32_t f0 = (lo + 15u) >> 4, f1 = hi >> 4;  // whole chunks [f0, f1)
  if (f1 > f0) {
    u32x4 v[kMax];
#pragma unroll
    for (int k = 0; k < kMax; k++) {
      const uint32_t c = min(f0 + (uint32_t)lane + (uint32_t)(kWave * k), f1 - 1u);
      v[k] = *(const u32x4 *)(lds + (c << 4));
    }
#pragma unroll
    for (int k = 0; k < kMax; k++) {
      const uint32_t c = f0 + (uint32_t)lane + (uint32_t)(kWave * k);
      if (c < f1) __builtin_nontemporal_store(v[k], (u32x4 *)(o_al + (c << 4)));
    }
  }
  const uint32_t head_end = min(hi, f0 << 4), tail_start = max(head_end, f1 << 4);
  const uint32_t x = lane < 16 ? lo + (uint32_t)lane : tail_start + (uint32_t)lane - 16u;
  if (lane < 32 && x < (lane < 16 ? head_end : hi)) o_al[x] = lds[x];
}

__device__ __forceinline__ uint32_t lds_byte(const uint32_t *w, uint32_t x) {
  return (w[x >> 2] >> ((x & 3u) * 8u)) & 0xffu;
}

int device_cus();

#ifndef MHQ_PER_CU  // workgroups per CU in a tile grid (waves then loop over tiles)
#define MHQ_PER_CU 1
#endif
// Persistent-style grid: at most `per_cu` workgroups per CU, never more than
// the tiles need.
inline unsigned tile_grid(uint64_t ntiles, int waves, int per_cu) {
  const uint64_t want = (ntiles + waves - 1) / waves;
  const uint64_t cap = (uint64_t)device_cus() * per_cu;
  return (unsigned)(want < cap ? want : cap);
}


// ---- read_strings' framed strings (str_frame.hip; finished in the decode) --
// kind: 0 raw, 1 Huffman, 2 header error (hc/io.go:74-81 return ("", nil)),
// | kDeclared when the declared length is not 0.
constexpr uint8_t kDeclared = 4;
// A framed string's output region in the positional layout: floor(8 x / 5)
// of its payload start x, without overflow (str_frame.hip).
__device__ __forceinline__ uint64_t region_at(uint64_t x) { return x / 5u * 8u + (x % 5u) * 8u / 5u; }
// A string's output capacity, recomputed from its parse where it is needed
// (the fallback layout, a cut region): floor(8*take/5) (Huffman), take (raw).
__device__ __forceinline__ uint64_t read_cap(uint8_t kind, uint64_t start, uint32_t hend, uint64_t next) {
  const uint32_t k = kind & 3u;
  if (k == 1u) return (uint32_t)((uint64_t)(uint32_t)(hend - (uint32_t)start) * 8u / 5u);
  return k == 0u ? (uint32_t)(next - start) : 0u;
}

// len bytes from src to dst, any alignments, by one thread: the 0-3 bytes up
// to dst's first dword boundary and the 0-3 after its last whole dword go as
// bytes (neighbouring bytes untouched), the middle as dword stores of source
// dwords realigned with v_alignbyte.  Every load of a 64-byte block is issued
// before its first store (no load-store round trip per word).  A source dword
// read holds at least one byte of [src, src + len): inside any 4-B aligned
// allocation.
__device__ __forceinline__ void copy_bytes(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
                                           uint64_t len) {
  const uint32_t h = (uint32_t)min((uint64_t)((0u - (uint32_t)(uintptr_t)dst) & 3u), len);
  const uint64_t body = (len - h) & ~(uint64_t)3;
  const uint32_t t = (uint32_t)(len - h) & 3u;
  CRUMB(41, src + len - 1);
  CRUMB(42, dst + len - 1);
  uint32_t hb[3], tb[3];
#pragma unroll
  for (uint32_t k = 0; k < 3; k++) {
    hb[k] = k < h ? src[k] : 0u;
    tb[k] = k < t ? src[h + body + k] : 0u;
  }
  const uint8_t *s1 = src + h;
  uint32_t *d4 = (uint32_t *)(dst + h);
  const uint32_t r = (uint32_t)(uintptr_t)s1 & 3u;
  const uint32_t *w = (const uint32_t *)(s1 - r);
  const uint64_t nw = body >> 2;
  for (uint64_t q0 = 0; q0 < nw; q0 += 16) {
    const uint32_t nq = (uint32_t)min(nw - q0, (uint64_t)16);
    const uint32_t nload = nq + (r != 0u);
    uint32_t x[17];
#pragma unroll
    for (uint32_t j = 0; j < 17; j++) x[j] = j < nload ? w[q0 + j] : 0u;
#pragma unroll
    for (uint32_t j = 0; j < 16; j++)
      if (j < nq) d4[q0 + j] = __builtin_amdgcn_alignbyte(x[j + 1], x[j], r);
  }
#pragma unroll
  for (uint32_t k = 0; k < 3; k++) {
    if (k < h) dst[k] = (uint8_t)hb[k];
    if (k < t) dst[h + body + k] = (uint8_t)tb[k];
  }
}

}  // namespace dev
}  // namespace mhq
