// huff_decode_stream.hip -- gfx950 batch decode of RFC 7541 Huffman literals,
// streamed: no tiles, no sort, no per-tile phases.
//
// Semantics: hc/huffman.go:102-121 (HuffmanDecompressor.Read) driven to EOF as
// Reader.ReadString does (hc/io.go:85-96), exactly as decode_kernel
// (huff_decode.hip) and the CPU oracle (oracle/huff_oracle.c).
//
// Why: the tile decode (huff_decode.hip) spends a third of its time outside
// the probe loop -- every wave stages, flushes, zeroes and sorts a tile, then
// loops, in lockstep with the other waves of its SIMD, and the first loop
// starts 6 us into the launch (DESIGN.md §4, round 5 timeline).  Here the
// probe loop never waits for memory:
//
//   * one workgroup per CU, 16 waves: 12 DECODERS and 4 LOADERS;
//   * decoder d owns a contiguous run of the workgroup's literals and three
//     LDS rings: input (4 KiB of byte-swapped stream words + a mirror of the
//     ring's first 272 bytes past its end, so a literal that wraps is read
//     contiguously), output (4 KiB in the global layout + 400 B of slack past
//     its end for the region that wraps) and the offsets of the literals in
//     flight (pin / pout: positions relative to the run's 16-B aligned bases)
//     with their results (lens);
//   * each lane decodes ONE literal at a time with the tile decode's masked
//     probe steps (win_pair / win_step32, groups of three steps) and, when it
//     finishes, records out_len | status in lens and goes idle; once kThr lanes
//     are idle the wave services them: the next literals in order go to the
//     idle lanes (a wave-uniform counter, mbcnt ranks: no atomics, no sort),
//     so lanes stay busy whatever the length mix (dynamic balance);
//   * the service also flushes the output ring up to the FRONTIER -- the
//     oldest literal still in flight (a DPP wave-min) -- as aligned 16-B
//     stores, zeroes what left, and stores out_len / status of the finished
//     literals below it (coalesced); the decoder issues stores only, never a
//     load, so nothing in its loop waits on vmcnt;
//   * loader l serves decoders l, l+4, l+8: it loads 1 KiB input chunks (and
//     64-entry offset chunks) into registers, waits, byte-swaps and writes
//     them into the rings and publishes how far each ring is staged
//     (in_staged, off_loaded, LDS words, release/acquire); it stages a chunk
//     only where the ring holds nothing at or after the decoder's published
//     frontier;
//   * literals the ring cannot take -- over 240 encoded bytes, an output
//     region over 384 bytes or one that can truncate (hc/huffman.go:104), and
//     malformed tails that decode a code across the literal's end (kSafe
//     steps pend nothing for them) -- are deferred: their region leaves the
//     ring as zeros and, once the run is flushed, the tile decode's streamed
//     long-literal path (decode_tile_long_body) decodes each exactly into
//     global memory.
//
// Ring invariants (positions are bytes from the run's aligned base, unwrapped;
// R = ring size, S = its slack):
//   input:  chunk c (bytes [1024c, 1024c+1024)) is written only when
//           1024(c+1) - pin[F] <= R, F the published frontier; a literal is
//           assigned only when pin[r+1] <= in_staged.
//   output: literal r is assigned only when pout[r+1] - out_flushed <= R - S,
//           so its ring positions (and the slack, which holds positions
//           [0, S) of the next lap) hold nothing unflushed; the flush of
//           positions [0, S) of a lap ORs the slack in.
//   offsets / lens: entry e lives at e % 256; an offsets chunk is written only
//           when it ends <= F + 256, a literal is assigned only when it is
//           < len_flushed + 256.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <cstring>

#include "huff_decode_dev.h"

namespace mhq {
namespace {

using namespace dev;

constexpr int kDecoders = 12;
constexpr int kLoaders = 4;
constexpr int kSWaves = kDecoders + kLoaders;
constexpr int kST = kSWaves * kWave;
static_assert(kDecoders % kLoaders == 0, "loader l serves decoders l, l + kLoaders, ...");
constexpr int kPerLoader = kDecoders / kLoaders;

constexpr uint32_t kRin = 4096;   // input ring (bytes, a multiple of the 1-KiB staging chunk)
constexpr uint32_t kSin = 256;    // longest literal the ring streams is kSin - 16 encoded bytes
constexpr uint32_t kMirror = kSin + 16;  // ring bytes [0, kMirror) are mirrored past its end
constexpr uint32_t kRout = 5120;  // output ring (bytes, a multiple of 16)
constexpr uint32_t kSout = 400;   // slack past it: the largest region the ring takes is kSout - 16
constexpr uint32_t kMaxIn = kSin - 16;
constexpr uint32_t kMaxOut = kSout - 16;
constexpr uint32_t kOffRing = 256;  // offsets / lens entries (power of two)
constexpr uint32_t kOffMask = kOffRing - 1;
constexpr uint32_t kChunk = 1024;   // input staging chunk: 64 lanes x 16 B
static_assert(kRin % kChunk == 0 && kRout % 16 == 0, "ring sizes");
constexpr uint32_t kDefMax = 16;    // deferred literals listed per decoder (more: the whole run again)
#ifndef MHQ_STREAM_GRAB
#define MHQ_STREAM_GRAB 80  // a lane takes its next literal when its current one has this many bits left
#endif
constexpr uint32_t kGrabBits = MHQ_STREAM_GRAB;
#ifndef MHQ_STREAM_FLUSH
#define MHQ_STREAM_FLUSH 256  // output bytes worth a flush before the run's end
#endif
constexpr uint32_t kFlushMin = MHQ_STREAM_FLUSH;
constexpr uint32_t kSpinMax = 1u << 22;  // bounded waits: a wedged ring ends the launch, not the GPU

struct alignas(16) DecRing {
  uint32_t in_w[(kRin + kMirror + 16) / 4];  // (+16: the steps' look-ahead words)
  uint32_t out_w[(kRout + kSout + 16) / 4];
  uint32_t pin[kOffRing];   // literal e's input start, bytes from the run's aligned input base
  uint32_t pout[kOffRing];  // its output region start, bytes from the aligned output base
  uint32_t in_staged;       // loader: input bytes [0, in_staged) are in the ring (or dead)
  uint32_t off_loaded;      // loader: offset entries [0, off_loaded) are in the ring
  uint32_t frontier;        // decoder: every literal below it is finished
  uint32_t loader_done;     // loader: nothing more will be written to this ring
  uint32_t ndef;
  uint32_t def[kDefMax];
};
static_assert(sizeof(uint32_t) * kLongWords * kWave <= sizeof(DecRing::in_w) + sizeof(DecRing::out_w),
              "the deferred literals' windows (decode_tile_long_body) fit the two rings");

struct StreamSmem {  // the tables at Smem's offsets (win_* take Smem)
  uint32_t lut1[kLut1Size];
  uint16_t lut2[kLut2Size];
  uint8_t clen[256];
  uint32_t next_tile;
  uint32_t abort;
  DecRing r[kDecoders];
};
static_assert(sizeof(StreamSmem) <= 163840, "one workgroup per CU");
static_assert(offsetof(StreamSmem, lut2) == offsetof(Smem, lut2) && offsetof(StreamSmem, clen) == offsetof(Smem, clen),
              "the step functions read the tables at Smem's offsets");

typedef __attribute__((address_space(3))) uint32_t lds_u32;

#ifdef MHQ_DIAG_STREAM
// Diagnostic build (-DMHQ_DIAG_STREAM): per wave counters of the last launch,
// g_sdiag[(block * 16 + wave) * kSDiag + k]; decoders: [0] cycles in run_all,
// [1] in service, [2] waiting for the loader, [3] services, [4] groups, [5]
// sum of active lanes over groups, [6] literals assigned, [7] flushes;
// loaders: [8] cycles, [9] iterations, [10] cycles in vmcnt waits, [11]
// chunks staged, [12] idle iterations.
constexpr int kSDiag = 16;
__device__ unsigned long long g_sdiag[1024 * 16 * kSDiag];
#define SDIAG_T0(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define SDIAG_ADD(k, x) (diag[(k)] += (unsigned long long)(x))
#define SDIAG_DECL unsigned long long diag[kSDiag] = {}
#define SDIAG_STORE()                                                                   \
  do {                                                                                  \
    if (lane == 0)                                                                      \
      for (int _k = 0; _k < kSDiag; _k++)                                               \
        g_sdiag[((uint64_t)blockIdx.x * 16 + threadIdx.x / kWave) * kSDiag + _k] = diag[_k]; \
  } while (0)
#else
#define SDIAG_T0(v) \
  do {              \
  } while (0)
#define SDIAG_ADD(k, x) \
  do {                  \
  } while (0)
#define SDIAG_DECL
#define SDIAG_STORE() \
  do {                \
  } while (0)
#endif

__device__ __forceinline__ uint32_t lds_acquire(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release(uint32_t *p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Minimum over the wave (every lane active), in DPP moves: prefix minima in
// rows of 16, then rows 1/3 and 2/3 take the lower rows' (as wave_incl_scan).
__device__ __forceinline__ uint32_t wave_min(uint32_t x) {
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x111, 0xf, 0xf, false));  // row_shr:1
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x112, 0xf, 0xf, false));  // row_shr:2
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x114, 0xf, 0xf, false));  // row_shr:4
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x118, 0xf, 0xf, false));  // row_shr:8
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x142, 0xa, 0xf, false));  // row_bcast:15
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}


// A decoder's run: literals [s, s + nlit); its input from the 16-B aligned
// ia16 (the run's first byte at idelta), its output regions from oa16.
struct Run {
  uint64_t s;
  uint32_t nlit;
  const uint8_t *ia16;
  uint8_t *oa16;
  uint32_t idelta, odelta, in_total, out_total;  // in_total / out_total: bytes from the aligned bases
  uint32_t ib32, ob32;                             // low words of in_off[s], out_off[s]
  bool bypass;  // spans of 2^31 bytes or more: the run goes through the long-literal path
  __device__ __forceinline__ void init(const uint8_t *in, const uint64_t *in_off, uint64_t in_bias, uint8_t *out,
                                       const uint64_t *out_off, uint64_t out_bias, uint64_t s_, uint32_t n_) {
    s = s_;
    nlit = n_;
    const uint64_t ib = in_off[s], ie = in_off[s + n_], ob = out_off[s], oe = out_off[s + n_];
    const uint8_t *ia = in + (ib - in_bias);
    uint8_t *oa = out + (ob - out_bias);
    idelta = (uint32_t)((uintptr_t)ia & 15u);
    odelta = (uint32_t)((uintptr_t)oa & 15u);
    ia16 = ia - idelta;
    oa16 = oa - odelta;
    ib32 = (uint32_t)ib;
    ob32 = (uint32_t)ob;
    bypass = ie < ib || oe < ob || ie - ib >= (1ull << 31) - 64 || oe - ob >= (1ull << 31) - 64;
    in_total = bypass ? 0u : (uint32_t)(ie - ib) + idelta;
    out_total = bypass ? 0u : (uint32_t)(oe - ob) + odelta;
  }
};

// ---------------------------------------------------------------- decoder --
struct Decoder {
  const StreamSmem &sm;
  DecRing &R;
  const Run &run;
  uint32_t *__restrict__ out_len;
  uint8_t *__restrict__ status;
  uint32_t lane;
  // wave-uniform
  uint32_t next_r = 0;       // the run's literals from next_r on are not handed out
  uint32_t out_flushed = 0;  // output ring positions below it are flushed (and zeroed)
  uint32_t tgt = 0;          // ... and those below it are final
  uint32_t ndef = 0;         // deferred literals listed in R.def
  // the loader's counters, read at the end of a group end for the next one
  // (stale by a group: conservative, they only grow)
  uint32_t off_ld = 0, in_st = 0;
  // the flush in flight: ring chunks [fl_lo, fl_hi) were read at the last
  // group end (one per lane at most: fv, with the slack's fs); they leave
  // (stores, zeroing) at this one
  uint32_t fl_lo = 0, fl_hi = 0;
  u32x4 fv = {0u, 0u, 0u, 0u}, fs = {0u, 0u, 0u, 0u};
  // per lane: the literal being decoded (cur)
  bool active = false, crossed = false;
  uint32_t r = 0, ost = 0, bc = 0;  // bc: cur's region start (unwrapped ring position)
  uint32_t cr = 0;                  // the literal that crossed its end in the last group
  WinBuf3 win;
  OutAccL acc;
  PendL pend;
  // per lane: the next literal.  stage 2: index j handed out and its ring
  // entries a0, a1 (input), b0, b1 (output) requested at the last group end;
  // stage 3: set up, every ring gate passed -- the lane moves to it when cur
  // ends, in place within the group.
  uint32_t stage = 0, j = 0, a0 = 0, a1 = 0, b0 = 0, b1 = 0, pm2 = 0, ost2 = 0;
  int32_t left2 = 0;
  SDIAG_DECL;

  __device__ Decoder(const StreamSmem &sm_, DecRing &R_, const Run &run_, uint32_t *ol, uint8_t *st, uint32_t lane_)
      : sm(sm_), R(R_), run(run_), out_len(ol), status(st), lane(lane_) {
    out_flushed = tgt = fl_lo = fl_hi = run.odelta;
    pend.p = R.out_w;
    pend.v = 0;
  }

  __device__ __forceinline__ void start_next() {
    r = j;
    win.pm = pm2;
    win.left = left2;
    win.set_mask();
    ost = ost2;
    bc = b0;
    acc.init(R.out_w, ost2);
    stage = 0;
    active = true;
  }

  // Three masked steps on the active lanes; a literal that ends stores its
  // out_len / status (the lanes of a group end near each other: a group's
  // stores touch a few lines) and its lane moves to the next literal if that
  // is ready.
  __device__ __forceinline__ void group() {
    bool stop;
    win_pair<false, true>((const Smem &)sm, win, acc, pend, stop);
    const bool fin = win_step32<true, true>((const Smem &)sm, win, acc, pend, stop);
    if (fin) {
      atomicOr(pend.p, pend.v);  // the literal's last word, before any flush can take its region
      pend.v = 0;
      crossed = win.left < 0;  // a code across the end: deferred at the group end (nothing of it was pended)
      cr = r;
      if (!crossed) {
        out_len[run.s + r] = acc.optr(R.out_w) - ost;
        status[run.s + r] = (uint8_t)(win.left > kEosOnes);
      }
      if (stage == 3u)
        start_next();
      else
        active = false;
    }
  }

  // Lanes whose `d` is set append `idx` to the deferred list (ranks by ballot:
  // no atomics, no round trip).
  __device__ __forceinline__ void defer_lanes(bool d, uint32_t idx) {
    const uint64_t m = __ballot(d);
    if (!m) return;
    const uint32_t k = ndef + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (d && k < kDefMax) R.def[k] = idx;
    ndef += popc64(m);
  }

  // Every lane, once per group: the frontier (the lowest literal a lane
  // holds, or next_r), the flush below it, then one step of each lane's fetch
  // of its next literal.  Nothing here waits for an LDS round trip: what it
  // reads from LDS was requested at the last group end, and the group's own
  // probe waits have drained it.  Returns the frontier.
  __device__ uint32_t group_end() {
    const uint32_t mine = min(active ? r : 0xffffffffu, stage >= 2u ? j : 0xffffffffu);
    const uint32_t F = min(wave_min(mine), next_r);
    // the output below the frontier literal's region (its 16-B chunk stays):
    // the lane holding that literal knows where its region starts
    if (F >= run.nlit) {
      tgt = run.out_total;
    } else {
      const uint64_t at = __ballot(mine == F);
      if (at) {
        const uint32_t st = (uint32_t)__builtin_amdgcn_readlane((int)(active && r == F ? bc : b0),
                                                              (int)__builtin_ctzll(at));
        tgt = max(tgt, st & ~15u);
      }
    }
    // the flush read at the last group end leaves; the next piece is read
    if (fl_hi > fl_lo) {
      const uint32_t c = (fl_lo >> 4) + lane;
      if (c < ((fl_hi + 15u) >> 4)) {
        const uint32_t q = (c << 4) % kRout;
        const u32x4 v = fv | fs;
        const uint32_t a = c << 4;
        uint8_t *g = run.oa16 + a;
        if (a >= fl_lo && a + 16u <= fl_hi) {
          __builtin_nontemporal_store(v, (u32x4 *)g);
        } else {  // the run's partial first / last chunk
          const uint32_t x0 = max(fl_lo, a) - a, x1 = min(fl_hi, a + 16u) - a;
          for (uint32_t x = x0; x < x1; x++) g[x] = (uint8_t)(v[x >> 2] >> (8u * (x & 3u)));
        }
        *(u32x4 *)(R.out_w + (q >> 2)) = u32x4{0u, 0u, 0u, 0u};
        if (q < kSout) *(u32x4 *)(R.out_w + ((kRout + q) >> 2)) = u32x4{0u, 0u, 0u, 0u};
      }
      out_flushed = fl_hi;
    }
    fl_lo = fl_hi = out_flushed;
    if (tgt - out_flushed >= kFlushMin || (F >= run.nlit && tgt > out_flushed)) {
      SDIAG_ADD(7, 1);
      fl_hi = min(tgt, ((out_flushed >> 4) + (uint32_t)kWave) << 4);
      const uint32_t c = (fl_lo >> 4) + lane;
      if (c < ((fl_hi + 15u) >> 4)) {
        const uint32_t q = (c << 4) % kRout;
        fv = *(const u32x4 *)(R.out_w + (q >> 2));
        fs = q < kSout ? *(const u32x4 *)(R.out_w + ((kRout + q) >> 2)) : u32x4{0u, 0u, 0u, 0u};
      }
    }
    // deferrals: literals that crossed their end in the group
    defer_lanes(crossed, cr);
    crossed = false;
    // stage 2 -> 3: classify the literal whose entries came in, gate it on the rings
    const uint32_t nb = a1 - a0, reg = b1 - b0;
    const bool s2 = stage == 2u;
    const bool empty = s2 && nb == 0u;
    const bool dfr = s2 && !empty && (a1 < a0 || b1 < b0 || nb > kMaxIn || reg > kMaxOut || reg < nb * 8u / 5u);
    if (empty) {
      out_len[run.s + j] = 0u;
      status[run.s + j] = 0;
    }
    defer_lanes(dfr, j);
    if (s2 && !empty && !dfr && a1 <= in_st && b1 - out_flushed <= kRout - kSout) {
      const uint32_t p0 = (a0 % kRin) * 8u;
      pm2 = 8u * (uint32_t)(uintptr_t)R.in_w + p0 - 1u;
      left2 = (int32_t)(nb * 8u);
      ost2 = b0 % kRout;
      stage = 3;
    }
    stage = (empty || dfr) ? 0u : stage;
    if (!active && stage == 3u) start_next();
    // new indices, in rank order, for the lanes that want one (idle, or cur
    // near its end); their entries are used at the next group end
    const bool want = stage == 0u && (!active || win.left <= (int32_t)kGrabBits);
    const uint64_t wm = __ballot(want);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(wm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)wm, 0u));
    const uint32_t avail = min(off_ld > next_r + 1u ? off_ld - 1u - next_r : 0u, run.nlit - next_r);
    const uint32_t na = min(popc64(wm), avail);
    if (want && rank < na) {
      j = next_r + rank;
      a0 = R.pin[j & kOffMask];
      a1 = R.pin[(j + 1u) & kOffMask];
      b0 = R.pout[j & kOffMask];
      b1 = R.pout[(j + 1u) & kOffMask];
      stage = 2;
    }
    next_r += na;
    if (lane == 0) __hip_atomic_store(&R.frontier, F, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    // the counters for the next group end (the loader's, read before any
    // entry they publish: LDS requests of a wave are served in order)
    asm volatile("" ::: "memory");
    off_ld = __hip_atomic_load(&R.off_loaded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    in_st = __hip_atomic_load(&R.in_staged, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return F;
  }

  __device__ void run_all() {
    uint32_t spins = 0;
    SDIAG_T0(t_start);
    while (true) {
      SDIAG_ADD(4, 1);
      SDIAG_ADD(5, popc64(__ballot(active)));
      if (active) group();
      SDIAG_T0(t_s);
      const uint32_t F = group_end();
      SDIAG_ADD(1, __builtin_amdgcn_s_memtime() - t_s);
      if (F >= run.nlit && out_flushed >= run.out_total && fl_hi == fl_lo) break;
      if (__ballot(active) == 0) {  // waiting for the loader, or for the fetch to refill
        if (++spins > kSpinMax || lds_acquire(&((StreamSmem &)sm).abort)) {
          lds_release(&((StreamSmem &)sm).abort, 1u);
          break;
        }
        SDIAG_ADD(3, 1);
        __builtin_amdgcn_s_sleep(1);
      } else {
        spins = 0;
      }
    }
    if (lane == 0) {
      R.ndef = ndef;
      lds_release(&R.frontier, run.nlit);
    }
    SDIAG_ADD(0, __builtin_amdgcn_s_memtime() - t_start);
    SDIAG_STORE();
  }
};

// ----------------------------------------------------------------- loader --
struct LoadState {
  uint32_t in_chunk, in_chunks, off_chunk, off_chunks;
  bool done;
};

__device__ __forceinline__ void put_swapped(uint32_t *w, u32x4 v) {
  v.x = __builtin_bswap32(v.x);
  v.y = __builtin_bswap32(v.y);
  v.z = __builtin_bswap32(v.z);
  v.w = __builtin_bswap32(v.w);
  *(u32x4 *)w = v;
}

__device__ void loader(StreamSmem &sm, const Run *runs, const uint64_t *__restrict__ in_off,
                       const uint64_t *__restrict__ out_off, uint32_t lw, uint32_t lane) {
  LoadState st[kPerLoader];
#pragma unroll
  for (int i = 0; i < kPerLoader; i++) {
    const Run &run = runs[i];
    st[i].in_chunk = 0;
    st[i].in_chunks = (run.in_total + kChunk - 1u) / kChunk;
    st[i].off_chunk = 0;
    st[i].off_chunks = run.nlit ? (run.nlit + 1u + kWave - 1u) / kWave : 0u;
    st[i].done = run.nlit == 0 || run.bypass;
    if (st[i].done && lane == 0) lds_release(&sm.r[lw + kLoaders * i].loader_done, 1u);
  }
  uint32_t spins = 0;
  SDIAG_DECL;
  SDIAG_T0(t_start);
  while (true) {
    SDIAG_ADD(9, 1);
    u32x4 tin[kPerLoader][2];
    uint32_t toi[kPerLoader][2], too[kPerLoader][2];
    uint32_t nin[kPerLoader], noff[kPerLoader];
    bool all_done = true;
#pragma unroll
    for (int i = 0; i < kPerLoader; i++) {
      nin[i] = noff[i] = 0;
      if (st[i].done) continue;
      all_done = false;
      DecRing &R = sm.r[lw + kLoaders * i];
      const Run &run = runs[i];
      const uint32_t F = __hip_atomic_load(&R.frontier, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      asm volatile("" ::: "memory");  // (in-order LDS: the entry read after the frontier is current)
      const uint32_t off_ld = min(st[i].off_chunk * (uint32_t)kWave, run.nlit + 1u);
      const uint32_t pinF = __builtin_amdgcn_readfirstlane(F < off_ld ? R.pin[F & kOffMask] : 0u);
      // chunks wholly below the frontier literal are dead: skip them
      st[i].in_chunk = max(st[i].in_chunk, min(pinF / kChunk, st[i].in_chunks));
      const uint32_t last16 = run.in_total ? (run.in_total - 1u) >> 4 : 0u;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint32_t c = st[i].in_chunk + (uint32_t)h;
        if (c < st[i].in_chunks && kChunk * (c + 1u) - pinF <= kRin) {
          nin[i] = h + 1;
          const uint32_t x = min(c * (kChunk / 16u) + lane, last16);
          tin[i][h] = __builtin_nontemporal_load((const u32x4 *)run.ia16 + x);
        }
      }
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint32_t kk = st[i].off_chunk + (uint32_t)h;
        if (kk < st[i].off_chunks && (uint32_t)kWave * (kk + 1u) - F <= kOffRing) {
          noff[i] = h + 1;
          const uint64_t e = run.s + min(kk * (uint32_t)kWave + lane, run.nlit);
          toi[i][h] = lo32(in_off, e);
          too[i][h] = lo32(out_off, e);
        }
      }
    }
    if (all_done) break;
    SDIAG_T0(t_v);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    SDIAG_ADD(10, __builtin_amdgcn_s_memtime() - t_v);
    bool progress = false;
#pragma unroll
    for (int i = 0; i < kPerLoader; i++) {
      if (st[i].done) continue;
      DecRing &R = sm.r[lw + kLoaders * i];
      const Run &run = runs[i];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        if ((uint32_t)h < nin[i]) {
          const uint32_t q = ((st[i].in_chunk + (uint32_t)h) % (kRin / kChunk)) * kChunk + 16u * lane;
          put_swapped(R.in_w + (q >> 2), tin[i][h]);
          if (q < kMirror) put_swapped(R.in_w + ((kRin + q) >> 2), tin[i][h]);
        }
        if ((uint32_t)h < noff[i]) {
          const uint32_t e = (st[i].off_chunk + (uint32_t)h) * (uint32_t)kWave + lane;
          if (e <= run.nlit) {
            R.pin[e & kOffMask] = toi[i][h] - run.ib32 + run.idelta;
            R.pout[e & kOffMask] = too[i][h] - run.ob32 + run.odelta;
          }
        }
      }
      SDIAG_ADD(11, nin[i]);
      st[i].in_chunk += nin[i];
      st[i].off_chunk += noff[i];
      progress = progress || nin[i] || noff[i];
      asm volatile("" ::: "memory");  // ring words first, then the counters that publish them
      if (lane == 0) {
        __hip_atomic_store(&R.in_staged, min(st[i].in_chunk * kChunk, run.in_total), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(&R.off_loaded, min(st[i].off_chunk * (uint32_t)kWave, run.nlit + 1u), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (st[i].in_chunk >= st[i].in_chunks && st[i].off_chunk >= st[i].off_chunks) {
        st[i].done = true;
        if (lane == 0) lds_release(&R.loader_done, 1u);
      }
    }
    if (!progress) {
      SDIAG_ADD(12, 1);
      if (++spins > kSpinMax || lds_acquire(&sm.abort)) {
        lds_release(&sm.abort, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    } else {
      spins = 0;
    }
  }
  SDIAG_ADD(8, __builtin_amdgcn_s_memtime() - t_start);
  SDIAG_STORE();
}

// The exact path for a decoder's deferred literals (after its run is flushed):
// decode_tile_long_body, one literal a call, windows in the decoder's rings.
__device__ void run_deferred(const StreamSmem &sm, DecRing &R, const Run &run, const uint8_t *__restrict__ in,
                             const uint64_t *__restrict__ in_off, uint64_t in_bias, uint8_t *__restrict__ out,
                             const uint64_t *__restrict__ out_off, uint64_t out_bias, uint32_t *__restrict__ out_len,
                             uint8_t *__restrict__ status, uint32_t lane) {
  const uint32_t nd = __builtin_amdgcn_readfirstlane(R.ndef);
  if (nd == 0 && !run.bypass) return;
  for (uint32_t sp = 0; !lds_acquire(&R.loader_done) && sp < kSpinMax; sp++) __builtin_amdgcn_s_sleep(2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's stores of these regions came first
  wave_sync();
  if (run.bypass || nd > kDefMax) {
    // the whole run, 64 literals a round (a batch of long literals: most of them deferred; the
    // literals the ring decoded are decoded again, to the same bytes)
    for (uint32_t x = 0; x < run.nlit; x += kWave)
      decode_tile_long_body<false, StreamSmem, DecRing, kLongWords>(sm, R, in, in_off, nullptr, in_bias, out, out_off,
                                                                  out_bias, out_len, status, run.s + x,
                                                                  min((uint32_t)kWave, run.nlit - x), lane);
    return;
  }
  for (uint32_t i = 0; i < nd; i++) {
    const uint32_t rr = __builtin_amdgcn_readfirstlane(R.def[i]);
    decode_tile_long_body<false, StreamSmem, DecRing, kLongWords>(sm, R, in, in_off, nullptr, in_bias, out, out_off,
                                                                out_bias, out_len, status, run.s + rr, 1u, lane);
  }
}

__global__ __launch_bounds__(kST) void decode_stream_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off, uint64_t in_bias, uint64_t n,
    uint8_t *__restrict__ out, const uint64_t *__restrict__ out_off, uint64_t out_bias, uint32_t *__restrict__ out_len,
    uint8_t *__restrict__ status, const uint32_t *__restrict__ g_lut1, const uint16_t *__restrict__ g_lut2,
    const uint8_t *__restrict__ g_len, uint64_t per_block) {
  __shared__ StreamSmem sm;
  const uint32_t tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
  const uint64_t L0 = (uint64_t)blockIdx.x * per_block;
  if (L0 >= n) return;
  const uint64_t L1 = min(L0 + per_block, n);
  static_assert(kLut1Size / 4 == kST && kLut2Size / 8 <= kST, "table copy shape");
  ((u32x4 *)sm.lut1)[tid] = ((const u32x4 *)g_lut1)[tid];
  if (tid < (uint32_t)(kLut2Size / 8)) ((u32x4 *)sm.lut2)[tid] = ((const u32x4 *)g_lut2)[tid];
  if (tid < 64u) ((uint32_t *)sm.clen)[tid] = ((const uint32_t *)g_len)[tid];
  if (tid == 0) sm.abort = 0;
  if (tid < (uint32_t)kDecoders) {
    DecRing &R = sm.r[tid];
    R.in_staged = 0;
    R.off_loaded = 0;
    R.frontier = 0;
    R.loader_done = 0;
    R.ndef = 0;
  }
  // the output rings start zeroed (the decode ORs into them)
  constexpr uint32_t kOutChunks = sizeof(DecRing::out_w) / 16u;
  for (uint32_t c = tid; c < kOutChunks * kDecoders; c += kST)
    ((u32x4 *)sm.r[c / kOutChunks].out_w)[c % kOutChunks] = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  const uint64_t per_dec = (L1 - L0 + kDecoders - 1) / kDecoders;
  if (wave < (uint32_t)kDecoders) {
    const uint64_t s = min(L0 + per_dec * wave, L1), e = min(s + per_dec, L1);
    Run run;
    run.init(in, in_off, in_bias, out, out_off, out_bias, s, (uint32_t)(e - s));
    DecRing &R = sm.r[wave];
    if (run.nlit && !run.bypass) {
      Decoder d(sm, R, run, out_len, status, lane);
      d.run_all();
    }
    if (run.nlit) run_deferred(sm, R, run, in, in_off, in_bias, out, out_off, out_bias, out_len, status, lane);
  } else {
    const uint32_t lw = wave - kDecoders;
    Run runs[kPerLoader];
#pragma unroll
    for (int i = 0; i < kPerLoader; i++) {
      const uint32_t d = lw + kLoaders * (uint32_t)i;
      const uint64_t s = min(L0 + per_dec * d, L1), e = min(s + per_dec, L1);
      runs[i].init(in, in_off, in_bias, out, out_off, out_bias, s, (uint32_t)(e - s));
    }
    loader(sm, runs, in_off, out_off, lw, lane);
  }
}

}  // namespace

namespace {
std::atomic<int> g_decode_form{-1};
}
int decode_form() {
  int f = g_decode_form.load(std::memory_order_relaxed);
  if (f < 0) {
    const char *e = getenv("MHQ_DECODE_FORM");
    f = e && !strcmp(e, "tile") ? kDecodeTile : (e && !strcmp(e, "stream") ? kDecodeStream : kDecodeAuto);
    int expect = -1;
    if (!g_decode_form.compare_exchange_strong(expect, f)) f = expect;
  }
  return f;
}
int set_decode_form(int form) {
  if (form < kDecodeAuto || form > kDecodeStream) return -1;
  const int prev = decode_form();
  g_decode_form.store(form);
  return prev;
}

#ifdef MHQ_DIAG_STREAM
extern "C" int mhq_diag_stream(unsigned long long *out, int n) {
  const int m = n < 1024 * 16 * kSDiag ? n : 1024 * 16 * kSDiag;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sdiag), m * sizeof(unsigned long long)) == hipSuccess ? kSDiag : -1;
}
#endif

// The streamed decode (no in_end); see the top of this file.  One workgroup
// per CU, each a contiguous range of at least 12 x 64 literals.
hipError_t launch_decode_stream(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                                uint64_t n, uint8_t *out, const uint64_t *out_off, uint64_t out_bias,
                                uint32_t *out_len, uint8_t *status, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t cus = (uint64_t)dev::device_cus();
  const uint64_t per_block = std::max<uint64_t>((n + cus - 1) / cus, (uint64_t)kDecoders * kWave);
  const unsigned grid = (unsigned)((n + per_block - 1) / per_block);
  decode_stream_kernel<<<dim3(grid), dim3(kST), 0, s>>>(in, in_off, in_bias, n, out, out_off, out_bias, out_len,
                                                        status, t.lut1, t.lut2, t.len, per_block);
  return hipGetLastError();
}

}  // namespace mhq
