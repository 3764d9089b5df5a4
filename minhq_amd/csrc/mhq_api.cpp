// mhq_api.cpp -- the C ABI of libmhq_huff.so (include/mhq_huff.h).
//
// Host-memory entry points shard the batch across the context's devices by
// encoded bytes (literals are independent, no collective), one
// host thread per device.  A device's shard runs as a pipeline of chunks of
// about kChunkBytes on kPipe streams, each with its own staging buffers:
// chunk c's H2D copies, kernel and D2H copies go on stream c % kPipe, so one
// chunk's upload, another's kernel and a third's download overlap (stream
// order keeps a staging set from being reused before its chunk is done).
// Offsets are rebased with a per-chunk bias instead of being rewritten.
// Device-resident entry points only enqueue kernels on the caller's stream.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/mhq_huff.h"
#include "huff_kernels.h"
#include "huff_table.h"

namespace {

using mhq::DevTables;

int hip_rc(hipError_t e) { return e == hipSuccess ? MHQ_OK : MHQ_EHIP - (int)e; }

#define MHQ_TRY(expr)                        \
  do {                                       \
    hipError_t _e = (expr);                  \
    if (_e != hipSuccess) return hip_rc(_e); \
  } while (0)

struct Buffer {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t reserve(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 16);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

#ifndef MHQ_HOST_PIPE
#define MHQ_HOST_PIPE 4
#endif
#ifndef MHQ_HOST_CHUNK_MB  // encode / decode: outputs as large as the inputs, copies overlap best in small chunks
#define MHQ_HOST_CHUNK_MB 2
#endif
#ifndef MHQ_HOST_LEN_CHUNK_MB  // encode_len (16 MB: encode_len alone 16 -> 27 GiB/s, but a later decode 24 -> 5, unexplained)
#define MHQ_HOST_LEN_CHUNK_MB 2
#endif
constexpr int kPipe = MHQ_HOST_PIPE;  // streams (and staging sets) per device for host-memory calls
// input bytes per pipelined chunk (the environment's MHQ_HOST_CHUNK_MB /
// MHQ_HOST_LEN_CHUNK_MB override the built-in sizes: tuning and the
// host-path experiments of tools/hostpath.py)
uint64_t env_mb(const char *name, uint64_t dflt) {
  const char *e = getenv(name);
  const long v = e ? atol(e) : 0;
  return (v > 0 && v <= 1024 ? (uint64_t)v : dflt) << 20;
}
const uint64_t kChunkBytes = env_mb("MHQ_HOST_CHUNK_MB", MHQ_HOST_CHUNK_MB);
const uint64_t kLenChunkBytes = env_mb("MHQ_HOST_LEN_CHUNK_MB", MHQ_HOST_LEN_CHUNK_MB);

struct Stage {
  hipStream_t s = nullptr;
  Buffer in, in_off, out, out_off, lens, status;
};

struct Device {
  int ordinal = 0;
  void *table_mem = nullptr;
  DevTables tables{};
  std::mutex mu;  // serialises host-memory calls (they share the staging buffers)
  hipStream_t stream = nullptr;
  Stage st[kPipe];
  // Scratch of the device-resident calls, one buffer per caller stream: work
  // on one stream runs in order, so a stream's buffer is reused without
  // synchronisation (no per-call hipMallocAsync/hipFreeAsync in the stream).
  struct Scratch {
    hipStream_t s;
    void *p;
    size_t bytes;
    int holders;  // callers between stream_scratch and the end of their enqueueing (ScratchLease)
    uint32_t tag = 0;  // the slots pool: the last look-back tag handed out on this buffer
  };
  std::mutex scratch_mu;
  std::vector<Scratch> scratch;
  // Look-back slots (mhq_huff_encode_packed_dev), one buffer per caller
  // stream, written by nothing else: a stale slot holds an earlier call's
  // tag, never another entry point's data.
  std::vector<Scratch> slots;
  // Buffers a stream outgrew.  Work queued (possibly by another thread on the
  // same stream) may still use them: once the last caller holding one has
  // finished enqueueing (its ScratchLease ends) an event is recorded on the
  // stream, and the buffer is freed when that event has completed (checked
  // whenever a scratch buffer is handed out or released), or at mhq_close.
  struct Retired {
    void *p;
    hipStream_t s;
    int holders;
    hipEvent_t done;  // recorded once holders reaches 0 (null before)
  };
  std::vector<Retired> retired;
};
constexpr size_t kMaxScratchStreams = 64;
constexpr size_t kMaxCachedWriteScratch = (size_t)64 << 20;

}  // namespace

struct mhq_ctx {
  std::vector<std::unique_ptr<Device>> devs;
};

namespace {

std::once_flag g_tables_once;
mhq::Tables g_tables;
bool g_tables_ok = false;

const mhq::Tables *tables() {
  std::call_once(g_tables_once, [] { g_tables_ok = mhq::build_tables(&g_tables); });
  return g_tables_ok ? &g_tables : nullptr;
}

int init_device(Device *d, int ordinal) {
  d->ordinal = ordinal;
  MHQ_TRY(hipSetDevice(ordinal));
  hipDeviceProp_t prop;
  MHQ_TRY(hipGetDeviceProperties(&prop, ordinal));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return MHQ_ENODEV;
  const mhq::Tables *t = tables();
  if (!t) return MHQ_EINVAL;
  const size_t sz = sizeof(t->code) + sizeof(t->len) + sizeof(t->lut1) + sizeof(t->lut2);
  MHQ_TRY(hipMalloc(&d->table_mem, sz));
  uint8_t *base = (uint8_t *)d->table_mem;
  // layout: lut1 | code | lut2 | len  (each naturally aligned)
  uint8_t *p_lut1 = base;
  uint8_t *p_code = p_lut1 + sizeof(t->lut1);
  uint8_t *p_lut2 = p_code + sizeof(t->code);
  uint8_t *p_len = p_lut2 + sizeof(t->lut2);
  MHQ_TRY(hipMemcpy(p_lut1, t->lut1, sizeof(t->lut1), hipMemcpyHostToDevice));
  MHQ_TRY(hipMemcpy(p_code, t->code, sizeof(t->code), hipMemcpyHostToDevice));
  MHQ_TRY(hipMemcpy(p_lut2, t->lut2, sizeof(t->lut2), hipMemcpyHostToDevice));
  MHQ_TRY(hipMemcpy(p_len, t->len, sizeof(t->len), hipMemcpyHostToDevice));
  d->tables.lut1 = (const uint32_t *)p_lut1;
  d->tables.code = (const uint32_t *)p_code;
  d->tables.lut2 = (const uint16_t *)p_lut2;
  d->tables.len = (const uint8_t *)p_len;
  MHQ_TRY(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
  for (Stage &x : d->st) MHQ_TRY(hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking));
  return MHQ_OK;
}

void free_device(Device *d) {
  (void)hipSetDevice(d->ordinal);
  for (Stage &x : d->st) {
    x.in.release();
    x.in_off.release();
    x.out.release();
    x.out_off.release();
    x.lens.release();
    x.status.release();
    if (x.s) (void)hipStreamDestroy(x.s);
  }
  if (d->stream) (void)hipStreamDestroy(d->stream);
  if (d->table_mem) (void)hipFree(d->table_mem);
  for (auto &x : d->scratch) (void)hipFree(x.p);
  d->scratch.clear();
  for (auto &x : d->slots) (void)hipFree(x.p);
  d->slots.clear();
  for (auto &r : d->retired) {
    (void)hipFree(r.p);
    if (r.done) (void)hipEventDestroy(r.done);
  }
  d->retired.clear();
}

// Records the event after which a retired buffer may be freed (no holder is
// left, so every use of it is already on the stream).  Under scratch_mu.
void mark_retired(Device::Retired &r) {
  if (r.holders > 0 || r.done) return;
  hipEvent_t ev = nullptr;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return;  // kept until mhq_close
  if (hipEventRecord(ev, r.s) != hipSuccess) {
    (void)hipEventDestroy(ev);
    return;
  }
  r.done = ev;
}

// Frees the retired buffers whose stream has passed its last use.  Under
// scratch_mu; called whenever a scratch buffer is handed out or released, so
// an outgrown buffer does not stay allocated until mhq_close.
void reap_retired(Device *d) {
  for (size_t i = 0; i < d->retired.size();) {
    Device::Retired &r = d->retired[i];
    if (r.done && hipEventQuery(r.done) == hipSuccess) {
      (void)hipFree(r.p);
      (void)hipEventDestroy(r.done);
      r = d->retired.back();
      d->retired.pop_back();
    } else {
      i++;
    }
  }
}

// The scratch buffer of stream s, at least `bytes` long, or null when the
// context already tracks kMaxScratchStreams streams (the caller then
// allocates in stream order).  A buffer that has to grow is replaced by a
// new one and the old one retired (freed by reap_retired once its stream has
// passed it): another thread may have just been handed it for work it is
// still queueing on the same stream.
void *stream_buffer(Device *d, std::vector<Device::Scratch> &pool, hipStream_t s, size_t bytes) {
  std::lock_guard<std::mutex> g(d->scratch_mu);
  reap_retired(d);
  for (auto &x : pool) {
    if (x.s != s) continue;
    if (x.bytes >= bytes) {
      x.holders++;
      return x.p;
    }
    size_t b = 1;
    while (b < bytes) b <<= 1;
    void *p = nullptr;
    if (hipMalloc(&p, b) != hipSuccess) return nullptr;
    d->retired.push_back(Device::Retired{x.p, s, x.holders, nullptr});
    mark_retired(d->retired.back());
    x.p = p;
    x.bytes = b;
    x.holders = 1;
    x.tag = 0;  // (the slots pool: a new buffer is zeroed before its first call)
    return x.p;
  }
  if (pool.size() >= kMaxScratchStreams) return nullptr;
  size_t b = 65536;
  while (b < bytes) b <<= 1;
  void *p = nullptr;
  if (hipMalloc(&p, b) != hipSuccess) return nullptr;
  pool.push_back(Device::Scratch{s, p, b, 1});
  return p;
}
void *stream_scratch(Device *d, hipStream_t s, size_t bytes) { return stream_buffer(d, d->scratch, s, bytes); }

// The packed encode's look-back slots for one call on stream s, and the
// call's tag (1 .. 2^30 - 1).  A slot whose tag equals the call's is taken
// as this call's, so the tags are per buffer and stream-ordered: a new
// buffer is zeroed (tag 0 is never handed out; a buffer replaced to grow
// starts over at 0 too), and when a buffer's tags wrap it is zeroed again in
// stream order before the call that restarts at 1 (ADVICE r5:
// stale slots of an older, larger call).
constexpr uint32_t kMaxSlotTag = (1u << 30) - 1u;
void *take_slots(Device *d, hipStream_t s, size_t bytes, uint32_t *tag) {
  void *p = stream_buffer(d, d->slots, s, bytes);
  if (!p) return nullptr;
  std::lock_guard<std::mutex> g(d->scratch_mu);
  for (auto &x : d->slots) {
    if (x.p != p) continue;
    if (x.tag == 0 || x.tag >= kMaxSlotTag) {
      if (hipMemsetAsync(p, 0, x.bytes, s) != hipSuccess) return nullptr;
      x.tag = 0;
    }
    *tag = ++x.tag;
    return p;
  }
  return nullptr;
}

// Ends a caller's hold on a buffer from stream_scratch (after it has
// enqueued every use of it).
void release_scratch(Device *d, void *p) {
  if (!p) return;
  std::lock_guard<std::mutex> g(d->scratch_mu);
  for (auto *pool : {&d->scratch, &d->slots})
    for (auto &x : *pool)
      if (x.p == p) {
        x.holders--;
        return;
      }
  for (auto &r : d->retired)
    if (r.p == p) {
      r.holders--;
      mark_retired(r);
      break;
    }
  reap_retired(d);
}

// stream_scratch for the lifetime of one ABI call.
struct ScratchLease {
  Device *d;
  void *p;
  ScratchLease(Device *d_, hipStream_t s, size_t bytes) : d(d_), p(bytes ? stream_scratch(d_, s, bytes) : nullptr) {}
  ScratchLease(Device *d_, std::vector<Device::Scratch> &pool, hipStream_t s, size_t bytes)
      : d(d_), p(bytes ? stream_buffer(d_, pool, s, bytes) : nullptr) {}
  ~ScratchLease() { release_scratch(d, p); }
  ScratchLease(const ScratchLease &) = delete;
  ScratchLease &operator=(const ScratchLease &) = delete;
};

Device *device(mhq_ctx *ctx, int dev) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return nullptr;
  return ctx->devs[dev].get();
}

// Splits [0,n) into ctx->devs.size() contiguous shards of near-equal bytes.
std::vector<uint64_t> shard_bounds(const uint64_t *off, uint64_t n, size_t parts) {
  std::vector<uint64_t> b(parts + 1, n);
  b[0] = 0;
  const uint64_t total = off[n] - off[0];
  for (size_t k = 1; k < parts; k++) {
    const uint64_t target = off[0] + (uint64_t)((unsigned __int128)total * k / parts);
    b[k] = (uint64_t)(std::lower_bound(off, off + n, target) - off);
    b[k] = std::max(b[k], b[k - 1]);
  }
  return b;
}

enum class Op { kEncodeLen, kEncode, kDecode };

struct HostJob {
  Op op;
  const uint8_t *in;
  const uint64_t *in_off;
  uint8_t *out;
  const uint64_t *out_off;
  uint32_t *lens;
  uint8_t *status;
};

// Enqueues literals [a, b) of a host-memory job on one stage's stream.
int run_chunk(Device *d, Stage &S, const HostJob &j, uint64_t a, uint64_t b) {
  const uint64_t m = b - a;
  if (m == 0) return MHQ_OK;
  hipStream_t s = S.s;
  const uint64_t in_bias = j.in_off[a];
  const uint64_t in_bytes = j.in_off[b] - j.in_off[a];
  MHQ_TRY(hipMemcpyAsync(S.in.p, j.in + (j.in_off[a] - j.in_off[0]), in_bytes, hipMemcpyHostToDevice, s));
  MHQ_TRY(hipMemcpyAsync(S.in_off.p, j.in_off + a, (m + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  const uint8_t *din = (const uint8_t *)S.in.p;
  const uint64_t *din_off = (const uint64_t *)S.in_off.p;
  if (j.op == Op::kEncodeLen) {
    MHQ_TRY(mhq::launch_encode_len(d->tables, din, din_off, in_bias, m, (uint32_t *)S.lens.p, s));
    return hip_rc(hipMemcpyAsync(j.lens + a, S.lens.p, m * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  }
  const uint64_t out_bias = j.out_off[a];
  const uint64_t out_bytes = j.out_off[b] - j.out_off[a];
  MHQ_TRY(hipMemcpyAsync(S.out_off.p, j.out_off + a, (m + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  // The staging region is zeroed first: it is copied back whole, and bytes
  // the kernels leave alone -- past a literal's out_len (decode), past its
  // enc_len in a region longer than that or of a literal the encode skips
  // (mhq_huff.h lets a region be longer) -- would otherwise carry an earlier
  // call's data, perhaps another request's headers, into the caller's
  // buffer.  The fill is in stream order, before the kernel (a few MB per
  // chunk, beside its PCIe copies).
  uint8_t *dout = (uint8_t *)S.out.p;
  MHQ_TRY(hipMemsetAsync(dout, 0, out_bytes, s));
  const uint64_t *dout_off = (const uint64_t *)S.out_off.p;
  if (j.op == Op::kEncode) {
    MHQ_TRY(mhq::launch_encode(d->tables, din, din_off, in_bias, m, dout, dout_off, out_bias, s));
  } else {
    MHQ_TRY(mhq::launch_decode(d->tables, din, din_off, in_bias, m, dout, dout_off, out_bias,
                               (uint32_t *)S.lens.p, (uint8_t *)S.status.p, s, nullptr, nullptr,
                               j.in_off[b] - j.in_off[a]));
    MHQ_TRY(hipMemcpyAsync(j.lens + a, S.lens.p, m * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    MHQ_TRY(hipMemcpyAsync(j.status + a, S.status.p, m, hipMemcpyDeviceToHost, s));
  }
  return hip_rc(
      hipMemcpyAsync(j.out + (j.out_off[a] - j.out_off[0]), dout, out_bytes, hipMemcpyDeviceToHost, s));
}

#ifndef MHQ_HOST_ZERO_COPY  // 0: host-memory calls always stage through device buffers
#define MHQ_HOST_ZERO_COPY 1
#endif
// Bytes past an input buffer's end that must lie in its mapping before a
// kernel reads it in place: the kernels read aligned 16-B chunks holding a
// valid byte (never a chunk wholly past the end), so 16 would do; 64 is
// margin.  Outputs need none: the kernels write exactly their regions.
constexpr uint64_t kZcSlack = 64;

// The device's view of host memory [p, p + len) when it lies in one pinned
// allocation the device maps (hipHostMalloc, torch's pin_memory) with
// `slack` bytes after it, else null (pageable memory, hipHostRegister'ed
// ranges whose extent the runtime does not report, buffers at a mapping's
// very end: those go through the staged copies).
const void *zero_copy_view(int ordinal, const void *p, uint64_t len, uint64_t slack = kZcSlack) {
  if (!p) return nullptr;
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) != hipSuccess || at.type != hipMemoryTypeHost || !at.devicePointer) {
    (void)hipGetLastError();  // (pageable memory reports an error: not the caller's)
    return nullptr;
  }
  // only memory pinned while this shard's device was current: a mapping
  // into the other devices of a multi-device context is not assumed
  if (at.device != ordinal) return nullptr;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) != hipSuccess || !base) {
    (void)hipGetLastError();
    return nullptr;
  }
  const uintptr_t b0 = (uintptr_t)base, x = (uintptr_t)p;
  if (b0 % 4096u) return nullptr;
  const uint64_t mapped = ((uint64_t)size + 4095u) & ~(uint64_t)4095u;  // pinned pages are mapped whole
  if (x < b0 || x - b0 + len + slack > mapped) return nullptr;
  return at.devicePointer;
}

// A host-memory job run in place: every buffer the op touches is pinned and
// mapped, so the kernels read and write it over PCIe with no staging copies
// (one launch per device shard).  Returns false (nothing enqueued) otherwise.
bool run_zero_copy(Device *d, const HostJob &j, uint64_t a, uint64_t b, int &rc) {
  if (!MHQ_HOST_ZERO_COPY) return false;
  const uint64_t m = b - a;
  const uint64_t n_all_in = j.in_off[b] - j.in_off[0];  // the view must reach the shard's end
  const uint8_t *din = (const uint8_t *)zero_copy_view(d->ordinal, j.in, n_all_in ? n_all_in : 1);
  const uint64_t *din_off = (const uint64_t *)zero_copy_view(d->ordinal, j.in_off + a, (m + 1) * sizeof(uint64_t));
  if (!din || !din_off) return false;
  hipStream_t s = d->st[0].s;
  if (j.op == Op::kEncodeLen) {
    uint32_t *dl = (uint32_t *)zero_copy_view(d->ordinal, j.lens + a, m * sizeof(uint32_t), 0);
    if (!dl) return false;
    rc = hip_rc(mhq::launch_encode_len(d->tables, din, din_off, j.in_off[0], m, dl, s));
  } else {
    const uint64_t n_all_out = j.out_off[b] - j.out_off[0];
    uint8_t *dout = (uint8_t *)zero_copy_view(d->ordinal, j.out, n_all_out ? n_all_out : 1, 0);
    const uint64_t *dout_off = (const uint64_t *)zero_copy_view(d->ordinal, j.out_off + a, (m + 1) * sizeof(uint64_t));
    if (!dout || !dout_off) return false;
    if (j.op == Op::kEncode) {
      rc = hip_rc(mhq::launch_encode(d->tables, din, din_off, j.in_off[0], m, dout, dout_off, j.out_off[0], s));
    } else {
      uint32_t *dl = (uint32_t *)zero_copy_view(d->ordinal, j.lens + a, m * sizeof(uint32_t), 0);
      uint8_t *dst = (uint8_t *)zero_copy_view(d->ordinal, j.status + a, m, 0);
      if (!dl || !dst) return false;
      rc = hip_rc(mhq::launch_decode(d->tables, din, din_off, j.in_off[0], m, dout, dout_off, j.out_off[0], dl, dst,
                                     s, nullptr, nullptr, j.in_off[a + m] - j.in_off[a]));
    }
  }
  const int r = hip_rc(hipStreamSynchronize(s));
  if (rc == MHQ_OK) rc = r;
  return true;
}

// Runs literals [a, b) of a host-memory job on one device: in place when the
// buffers allow (run_zero_copy), else in chunks of about kChunkBytes of input
// (kLenChunkBytes for encode_len), pipelined over the device's kPipe stages.
int run_shard(Device *d, const HostJob &j, uint64_t a, uint64_t b) {
  const uint64_t m = b - a;
  if (m == 0) return MHQ_OK;
  std::lock_guard<std::mutex> lock(d->mu);
  MHQ_TRY(hipSetDevice(d->ordinal));
  {
    int zrc = MHQ_OK;
    if (run_zero_copy(d, j, a, b, zrc)) return zrc;
  }
  const uint64_t in_bytes = j.in_off[b] - j.in_off[a];
  const uint64_t chunk = j.op == Op::kEncodeLen ? kLenChunkBytes : kChunkBytes;
  const size_t nch = (size_t)std::max<uint64_t>(1, std::min<uint64_t>(m, (in_bytes + chunk - 1) / chunk));
  std::vector<uint64_t> cb = shard_bounds(j.in_off + a, m, nch);
  // staging sized for the largest chunk, before anything is enqueued
  uint64_t max_m = 0, max_in = 0, max_out = 0;
  for (size_t c = 0; c < nch; c++) {
    const uint64_t x = a + cb[c], y = a + cb[c + 1];
    max_m = std::max(max_m, y - x);
    max_in = std::max(max_in, j.in_off[y] - j.in_off[x]);
    if (j.op != Op::kEncodeLen) max_out = std::max(max_out, j.out_off[y] - j.out_off[x]);
  }
  const int used = (int)std::min<size_t>(nch, kPipe);
  for (int k = 0; k < used; k++) {
    Stage &S = d->st[k];
    MHQ_TRY(S.in.reserve(max_in + 16));
    MHQ_TRY(S.in_off.reserve((max_m + 1) * sizeof(uint64_t)));
    MHQ_TRY(S.lens.reserve(max_m * sizeof(uint32_t)));
    if (j.op != Op::kEncodeLen) {
      MHQ_TRY(S.out.reserve(max_out + 16));
      MHQ_TRY(S.out_off.reserve((max_m + 1) * sizeof(uint64_t)));
      MHQ_TRY(S.status.reserve(max_m));
    }
  }
  int rc = MHQ_OK;
#ifdef MHQ_X_HOSTPROF  // (host-path experiment: enqueue and wait times per call, on stderr)
  const auto t0 = std::chrono::steady_clock::now();
  double worst = 0;
  for (size_t c = 0; c < nch && rc == MHQ_OK; c++) {
    const auto c0 = std::chrono::steady_clock::now();
    rc = run_chunk(d, d->st[c % kPipe], j, a + cb[c], a + cb[c + 1]);
    worst = std::max(worst, std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c0).count());
  }
  const auto t1 = std::chrono::steady_clock::now();
#else
  for (size_t c = 0; c < nch && rc == MHQ_OK; c++) rc = run_chunk(d, d->st[c % kPipe], j, a + cb[c], a + cb[c + 1]);
#endif
  for (int k = 0; k < used; k++) {
    const int r = hip_rc(hipStreamSynchronize(d->st[k].s));
    if (rc == MHQ_OK) rc = r;
  }
#ifdef MHQ_X_HOSTPROF
  const auto t2 = std::chrono::steady_clock::now();
  fprintf(stderr, "hostprof op=%d chunks=%zu enqueue_us=%.0f worst_chunk_us=%.0f wait_us=%.0f\n", (int)j.op, nch,
          std::chrono::duration<double, std::micro>(t1 - t0).count(), worst,
          std::chrono::duration<double, std::micro>(t2 - t1).count());
#endif
  return rc;
}

int run_host(mhq_ctx *ctx, const HostJob &j, uint64_t n) {
  if (!ctx || ctx->devs.empty()) return MHQ_EINVAL;
  if (n == 0) return MHQ_OK;
  if (!j.in_off || (!j.in && j.in_off[n] != j.in_off[0])) return MHQ_EINVAL;
  const size_t D = ctx->devs.size();
  std::vector<uint64_t> b = shard_bounds(j.in_off, n, D);
  if (D == 1) return run_shard(ctx->devs[0].get(), j, 0, n);
  std::vector<int> rc(D, MHQ_OK);
  std::vector<std::thread> th;
  for (size_t k = 0; k < D; k++)
    th.emplace_back([&, k] { rc[k] = run_shard(ctx->devs[k].get(), j, b[k], b[k + 1]); });
  for (auto &t : th) t.join();
  for (int r : rc)
    if (r != MHQ_OK) return r;
  return MHQ_OK;
}

}  // namespace

extern "C" {

int mhq_open(mhq_ctx **out, int ndev) {
  if (!out) return MHQ_EINVAL;
  *out = nullptr;
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count == 0) return MHQ_ENODEV;
  if (ndev <= 0 || ndev > count) ndev = count;
  std::vector<int> ord(ndev);
  for (int i = 0; i < ndev; i++) ord[i] = i;
  return mhq_open_devices(out, ord.data(), ndev);
}

int mhq_open_devices(mhq_ctx **out, const int *ordinals, int ndev) {
  if (!out || !ordinals || ndev <= 0) return MHQ_EINVAL;
  *out = nullptr;
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count == 0) return MHQ_ENODEV;
  auto ctx = std::make_unique<mhq_ctx>();
  for (int i = 0; i < ndev; i++) {
    if (ordinals[i] < 0 || ordinals[i] >= count) {
      for (auto &x : ctx->devs) free_device(x.get());
      return MHQ_EINVAL;
    }
    auto d = std::make_unique<Device>();
    int rc = init_device(d.get(), ordinals[i]);
    if (rc != MHQ_OK) {
      free_device(d.get());
      for (auto &x : ctx->devs) free_device(x.get());
      return rc;
    }
    ctx->devs.push_back(std::move(d));
  }
  *out = ctx.release();
  return MHQ_OK;
}

void mhq_close(mhq_ctx *ctx) {
  if (!ctx) return;
  for (auto &d : ctx->devs) free_device(d.get());
  delete ctx;
}

int mhq_device_count(const mhq_ctx *ctx) { return ctx ? (int)ctx->devs.size() : 0; }

const char *mhq_strerror(int rc) {
  switch (rc) {
    case MHQ_OK: return "ok";
    case MHQ_EINVAL: return "invalid argument";
    case MHQ_ENOMEM: return "out of memory";
    case MHQ_ENODEV: return "no gfx950 (MI355X) device available";
    default:
      if (rc <= MHQ_EHIP) return hipGetErrorString((hipError_t)(MHQ_EHIP - rc));
      return "unknown error";
  }
}

void *mhq_host_alloc(size_t bytes) {
  // kZcSlack more than asked: an input that ends where the caller's buffer
  // ends still has the slack the in-place route wants after it
  void *p = nullptr;
  if (hipHostMalloc(&p, bytes + kZcSlack, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}

void mhq_host_free(void *p) {
  if (p) (void)hipHostFree(p);
}

int mhq_code_table(uint8_t *len, uint32_t *code) {
  const mhq::Tables *t = tables();
  if (!t || !len || !code) return MHQ_EINVAL;
  memcpy(len, t->len, sizeof(t->len));
  memcpy(code, t->code, sizeof(t->code));
  return MHQ_OK;
}

int mhq_huff_encode_len(mhq_ctx *ctx, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                        uint32_t *enc_len) {
  if (n && !enc_len) return MHQ_EINVAL;
  return run_host(ctx, HostJob{Op::kEncodeLen, in, in_off, nullptr, nullptr, enc_len, nullptr}, n);
}

int mhq_huff_encode(mhq_ctx *ctx, const uint8_t *in, const uint64_t *in_off, uint64_t n, uint8_t *out,
                    const uint64_t *out_off) {
  if (n && (!out_off || (!out && out_off[n] != out_off[0]))) return MHQ_EINVAL;
  return run_host(ctx, HostJob{Op::kEncode, in, in_off, out, out_off, nullptr, nullptr}, n);
}

int mhq_huff_decode(mhq_ctx *ctx, const uint8_t *in, const uint64_t *in_off, uint64_t n, uint8_t *out,
                    const uint64_t *out_off, uint32_t *out_len, uint8_t *status) {
  if (n && (!out_off || !out_len || !status || (!out && out_off[n] != out_off[0]))) return MHQ_EINVAL;
  return run_host(ctx, HostJob{Op::kDecode, in, in_off, out, out_off, out_len, status}, n);
}

int mhq_huff_encode_len_dev(mhq_ctx *ctx, int dev, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                            uint32_t *enc_len, void *stream) {
  Device *d = device(ctx, dev);
  if (!d || (n && (!in_off || !enc_len))) return MHQ_EINVAL;
  MHQ_TRY(hipSetDevice(d->ordinal));
  return hip_rc(mhq::launch_encode_len(d->tables, in, in_off, 0, n, enc_len, (hipStream_t)stream));
}

int mhq_huff_offsets_dev(mhq_ctx *ctx, int dev, const uint32_t *enc_len, uint64_t n, uint64_t base,
                         uint64_t *out_off, uint64_t *cap_off, void *stream) {
  Device *d = device(ctx, dev);
  if (!d || !out_off || (n && !enc_len)) return MHQ_EINVAL;
  MHQ_TRY(hipSetDevice(d->ordinal));
  hipStream_t s = (hipStream_t)stream;
  ScratchLease scratch(d, s, mhq::offsets_scratch_bytes(n));
  return hip_rc(mhq::launch_offsets(enc_len, n, base, out_off, cap_off, s, scratch.p));
}

int mhq_huff_encode_layout_dev(mhq_ctx *ctx, int dev, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                               uint64_t base, uint32_t *enc_len, uint64_t *out_off, uint64_t *cap_off,
                               void *stream) {
  Device *d = device(ctx, dev);
  if (!d || !out_off || (n && (!in_off || !enc_len))) return MHQ_EINVAL;
  MHQ_TRY(hipSetDevice(d->ordinal));
  hipStream_t s = (hipStream_t)stream;
  const size_t bytes = mhq::offsets_sums_scratch_bytes(n);
  ScratchLease lease(d, s, bytes);
  uint64_t *sums = (uint64_t *)lease.p;
  const bool own = sums == nullptr;
  if (own) MHQ_TRY(hipMallocAsync((void **)&sums, bytes, s));
  hipError_t e = mhq::launch_encode_len(d->tables, in, in_off, 0, n, enc_len, s, sums);
  if (e == hipSuccess) e = mhq::launch_offsets_sums(enc_len, n, sums, base, out_off, cap_off, s);
  const hipError_t e2 = own ? hipFreeAsync(sums, s) : hipSuccess;
  return hip_rc(e != hipSuccess ? e : e2);
}

#ifndef MHQ_PK_MAX_MEAN  // the packed encode's largest mean literal (bytes)
#define MHQ_PK_MAX_MEAN 40
#endif
int mhq_huff_encode_packed_dev(mhq_ctx *ctx, int dev, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                               uint64_t in_bytes, uint64_t base, uint32_t *enc_len, uint64_t *out_off,
                               uint64_t *cap_off, uint8_t *out, uint64_t out_cap, void *stream) {
  Device *d = device(ctx, dev);
  if (!d || !out_off || (n && (!in_off || !enc_len || !out))) return MHQ_EINVAL;
  // every literal pads to whole bytes: sum ceil(30 L_i / 8) <= floor(30 in_bytes / 8) + n
  if (in_bytes > (UINT64_MAX - n) / 30 || out_cap < 30 * in_bytes / 8 + n) return MHQ_EINVAL;
  MHQ_TRY(hipSetDevice(d->ordinal));
  hipStream_t s = (hipStream_t)stream;
  // one launch for short literals (a mean <= 40 B: a range of 512 stages in 24 KB; and
  // every look-back sum under 2^32); otherwise the layout call and the
  // encode, whose forms suit long literals
  if (in_bytes < ((uint64_t)1 << 29) && in_bytes <= (uint64_t)MHQ_PK_MAX_MEAN * n) {
    uint32_t tag = 0;
    void *sp = take_slots(d, s, mhq::encode_packed_slot_bytes(n), &tag);
    if (sp) {
      const hipError_t e = mhq::launch_encode_packed(d->tables, in, in_off, 0, n, base, enc_len, out_off, cap_off,
                                                     out, out_cap, (uint64_t *)sp, tag, s, in_bytes);
      release_scratch(d, sp);
      return hip_rc(e);
    }
  }
  const int rc = mhq_huff_encode_layout_dev(ctx, dev, in, in_off, n, base, enc_len, out_off, cap_off, stream);
  if (rc != MHQ_OK || n == 0) return rc;
  // (launch_encode places literal i at out_off[i] - base from `out`)
  return hip_rc(mhq::launch_encode(d->tables, in, in_off, 0, n, out, out_off, base, s));
}

int mhq_huff_capacity_dev(mhq_ctx *ctx, int dev, const uint64_t *in_off, uint64_t n, uint64_t base,
                          uint64_t *cap_off, void *stream) {
  Device *d = device(ctx, dev);
  if (!d || !cap_off || !in_off) return MHQ_EINVAL;
  MHQ_TRY(hipSetDevice(d->ordinal));
  return hip_rc(mhq::launch_capacity(in_off, n, base, cap_off, (hipStream_t)stream));
}

int mhq_huff_encode_dev(mhq_ctx *ctx, int dev, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                        uint8_t *out, const uint64_t *out_off, void *stream) {
  Device *d = device(ctx, dev);
  if (!d || (n && (!in_off || !out_off))) return MHQ_EINVAL;
  MHQ_TRY(hipSetDevice(d->ordinal));
  return hip_rc(mhq::launch_encode(d->tables, in, in_off, 0, n, out, out_off, 0, (hipStream_t)stream));
}

int mhq_huff_decode_sized_dev(mhq_ctx *ctx, int dev, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                              uint64_t in_bytes, uint8_t *out, const uint64_t *out_off, uint32_t *out_len,
                              uint8_t *status, void *stream) {
  Device *d = device(ctx, dev);
  if (!d || (n && (!in_off || !out_off || !out_len || !status))) return MHQ_EINVAL;
  MHQ_TRY(hipSetDevice(d->ordinal));
  return hip_rc(mhq::launch_decode(d->tables, in, in_off, 0, n, out, out_off, 0, out_len, status,
                                   (hipStream_t)stream, nullptr, nullptr, in_bytes));
}

int mhq_set_decode_form(int form) {
  const int prev = mhq::set_decode_form(form);
  return prev < 0 ? MHQ_EINVAL : prev;
}

int mhq_debug_poison_scratch(int on) { return mhq::debug_poison_scratch.exchange(on ? 1 : 0); }

int mhq_huff_decode_dev(mhq_ctx *ctx, int dev, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                        uint8_t *out, const uint64_t *out_off, uint32_t *out_len, uint8_t *status,
                        void *stream) {
  return mhq_huff_decode_sized_dev(ctx, dev, in, in_off, n, 0, out, out_off, out_len, status, stream);
}

int mhq_read_strings_dev(mhq_ctx *ctx, int dev, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos,
                         const uint64_t *limit, const uint8_t *prefix, uint64_t n, uint8_t *out, uint64_t out_cap,
                         uint64_t *out_off, uint32_t *out_len, uint8_t *status, uint64_t *next, void *stream) {
  Device *d = device(ctx, dev);
  if (!d || !out_off || (n && (!blk || !pos || !limit || !prefix || !out || !out_len || !status || !next)))
    return MHQ_EINVAL;
  if (out_cap < blk_len / 5 * 8 + (blk_len % 5) * 8 / 5 + 1) return MHQ_EINVAL;
  MHQ_TRY(hipSetDevice(d->ordinal));
  hipStream_t s = (hipStream_t)stream;
  // the stream's cached scratch (null: the launcher allocates in stream order)
  ScratchLease lease(d, s, n ? mhq::read_strings_scratch_bytes(n, blk_len) : 0);
  void *scratch = n ? lease.p : nullptr;
  return hip_rc(mhq::launch_read_strings(d->tables, blk, blk_len, pos, limit, prefix, n, out, out_cap, out_off,
                                         out_len, status, next, s, scratch));
}

int mhq_write_strings_dev(mhq_ctx *ctx, int dev, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                          const uint8_t *prefix, const uint8_t *lead, int choice, uint8_t *out, uint64_t out_cap,
                          uint64_t *out_off, uint8_t *status, void *stream) {
  Device *d = device(ctx, dev);
  if (!d || !out_off || choice < MHQ_HUFF_AUTO || choice > MHQ_HUFF_NEVER) return MHQ_EINVAL;
  if (n && (!in_off || !prefix || !lead || (out && !status))) return MHQ_EINVAL;
  MHQ_TRY(hipSetDevice(d->ordinal));
  hipStream_t s = (hipStream_t)stream;
  // The scratch holds the packed Huffman payloads, bounded only by out_cap (no
  // size comes back to the host).  A scratch above kMaxCachedWriteScratch is
  // taken in stream order for this call (hipMallocAsync / hipFreeAsync)
  // rather than kept by the per-stream cache: a caller sizing out_cap for the
  // worst case must not pin that much device memory until mhq_close.
  const size_t want = mhq::write_strings_scratch_bytes(n, out ? out_cap : 0);
  ScratchLease lease(d, s, n && want <= kMaxCachedWriteScratch ? want : 0);
  void *scratch = n && want <= kMaxCachedWriteScratch ? lease.p : nullptr;
  return hip_rc(mhq::launch_write_strings(d->tables, in, in_off, n, prefix, lead, (uint32_t)choice, out, out_cap,
                                          out_off, status, s, scratch));
}

int mhq_read_ints_dev(mhq_ctx *ctx, int dev, const uint8_t *blk, const uint64_t *pos, const uint64_t *limit,
                      const uint8_t *prefix, uint64_t n, int index, uint64_t *value, uint64_t *next,
                      uint8_t *status, void *stream) {
  Device *d = device(ctx, dev);
  if (!d || (n && (!blk || !pos || !limit || !prefix || !value || !next || !status))) return MHQ_EINVAL;
  MHQ_TRY(hipSetDevice(d->ordinal));
  return hip_rc(mhq::launch_read_ints(blk, pos, limit, prefix, n, index, value, next, status, (hipStream_t)stream));
}

int mhq_write_ints_dev(mhq_ctx *ctx, int dev, const uint64_t *value, const uint8_t *prefix, const uint8_t *lead,
                       uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint8_t *status,
                       void *stream) {
  Device *d = device(ctx, dev);
  if (!d || !out_off || (n && (!value || !prefix || !lead || (out && !status)))) return MHQ_EINVAL;
  MHQ_TRY(hipSetDevice(d->ordinal));
  return hip_rc(
      mhq::launch_write_ints(value, prefix, lead, n, out, out_cap, out_off, status, (hipStream_t)stream));
}

int mhq_read_varints_dev(mhq_ctx *ctx, int dev, const uint8_t *blk, const uint64_t *pos, const uint64_t *limit,
                         uint64_t n, uint64_t *value, uint64_t *next, uint8_t *status, void *stream) {
  Device *d = device(ctx, dev);
  if (!d || (n && (!blk || !pos || !limit || !value || !next || !status))) return MHQ_EINVAL;
  MHQ_TRY(hipSetDevice(d->ordinal));
  return hip_rc(mhq::launch_read_varints(blk, pos, limit, n, value, next, status, (hipStream_t)stream));
}

int mhq_read_frames_dev(mhq_ctx *ctx, int dev, const uint8_t *blk, const uint64_t *pos, const uint64_t *limit,
                        uint64_t n, uint8_t *type, uint64_t *payload_len, uint64_t *payload_pos, uint8_t *status,
                        void *stream) {
  Device *d = device(ctx, dev);
  if (!d || (n && (!blk || !pos || !limit || !type || !payload_len || !payload_pos || !status))) return MHQ_EINVAL;
  MHQ_TRY(hipSetDevice(d->ordinal));
  return hip_rc(mhq::launch_read_frames(blk, pos, limit, n, type, payload_len, payload_pos, status,
                                        (hipStream_t)stream));
}

int mhq_write_varints_dev(mhq_ctx *ctx, int dev, const uint64_t *value, uint64_t n, uint8_t *out, uint64_t out_cap,
                          uint64_t *out_off, uint8_t *status, void *stream) {
  Device *d = device(ctx, dev);
  if (!d || !out_off || (n && (!value || (out && !status)))) return MHQ_EINVAL;
  MHQ_TRY(hipSetDevice(d->ordinal));
  return hip_rc(mhq::launch_write_varints(value, n, out, out_cap, out_off, status, (hipStream_t)stream));
}

}  // extern "C"

namespace {

template <class T>
struct DevArray {  // one call's device copy of a host array
  T *p = nullptr;
  ~DevArray() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(uint64_t count) { return hipMalloc((void **)&p, (count ? count : 1) * sizeof(T)); }
  hipError_t put(const T *src, uint64_t count, hipStream_t s) {
    hipError_t e = alloc(count);
    if (e == hipSuccess && count) e = hipMemcpyAsync(p, src, count * sizeof(T), hipMemcpyHostToDevice, s);
    return e;
  }
  hipError_t get(T *dst, uint64_t count, hipStream_t s) const {
    return count ? hipMemcpyAsync(dst, p, count * sizeof(T), hipMemcpyDeviceToHost, s) : hipSuccess;
  }
};

}  // namespace

extern "C" {

int mhq_read_strings(mhq_ctx *ctx, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos, const uint64_t *limit,
                     const uint8_t *prefix, uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *out_off,
                     uint32_t *out_len, uint8_t *status, uint64_t *next) {
  Device *d = device(ctx, 0);
  if (!d || !out_off || (n && (!blk || !pos || !limit || !prefix || !out || !out_len || !status || !next)))
    return MHQ_EINVAL;
  if (out_cap < blk_len / 5 * 8 + (blk_len % 5) * 8 / 5 + 1) return MHQ_EINVAL;
  for (uint64_t i = 0; i < n; i++)
    if (limit[i] > blk_len) return MHQ_EINVAL;
  std::lock_guard<std::mutex> lock(d->mu);
  MHQ_TRY(hipSetDevice(d->ordinal));
  hipStream_t s = d->stream;
  DevArray<uint8_t> dblk, dprefix, dout, dst;
  DevArray<uint64_t> dpos, dlim, doff, dnext;
  DevArray<uint32_t> dlen;
  MHQ_TRY(dblk.put(blk, blk_len, s));
  MHQ_TRY(dpos.put(pos, n, s));
  MHQ_TRY(dlim.put(limit, n, s));
  MHQ_TRY(dprefix.put(prefix, n, s));
  MHQ_TRY(dout.alloc(out_cap));
  MHQ_TRY(doff.alloc(n + 1));
  MHQ_TRY(dlen.alloc(n));
  MHQ_TRY(dst.alloc(n));
  MHQ_TRY(dnext.alloc(n));
  {
    // the per-stream scratch, as the device form takes it (no stream-ordered
    // allocation and free per call; without a cached buffer the launcher
    // allocates in stream order)
    ScratchLease lease(d, s, n ? mhq::read_strings_scratch_bytes(n, blk_len) : 0);
    MHQ_TRY(mhq::launch_read_strings(d->tables, dblk.p, blk_len, dpos.p, dlim.p, dprefix.p, n, dout.p, out_cap,
                                     doff.p, dlen.p, dst.p, dnext.p, s, lease.p));
  }
  MHQ_TRY(doff.get(out_off, n + 1, s));
  MHQ_TRY(hipStreamSynchronize(s));
  MHQ_TRY(dout.get(out, std::min<uint64_t>(out_off[n], out_cap), s));
  MHQ_TRY(dlen.get(out_len, n, s));
  MHQ_TRY(dst.get(status, n, s));
  MHQ_TRY(dnext.get(next, n, s));
  return hip_rc(hipStreamSynchronize(s));
}

int mhq_write_strings(mhq_ctx *ctx, const uint8_t *in, const uint64_t *in_off, uint64_t n, const uint8_t *prefix,
                      const uint8_t *lead, int choice, uint8_t *out, uint64_t out_cap, uint64_t *out_off,
                      uint8_t *status) {
  Device *d = device(ctx, 0);
  if (!d || !out_off || choice < MHQ_HUFF_AUTO || choice > MHQ_HUFF_NEVER) return MHQ_EINVAL;
  if (n && (!in_off || !prefix || !lead || (out && !status))) return MHQ_EINVAL;
  std::lock_guard<std::mutex> lock(d->mu);
  MHQ_TRY(hipSetDevice(d->ordinal));
  hipStream_t s = d->stream;
  const uint64_t base = n ? in_off[0] : 0, bytes = n ? in_off[n] - in_off[0] : 0;
  std::vector<uint64_t> rel(n + 1);
  for (uint64_t i = 0; i <= n; i++) rel[i] = n ? in_off[i] - base : 0;
  DevArray<uint8_t> din, dprefix, dlead, dout, dst;
  DevArray<uint64_t> doff, dout_off;
  MHQ_TRY(din.put(in, bytes, s));
  MHQ_TRY(doff.put(rel.data(), n + 1, s));
  MHQ_TRY(dprefix.put(prefix, n, s));
  MHQ_TRY(dlead.put(lead, n, s));
  MHQ_TRY(dout_off.alloc(n + 1));
  MHQ_TRY(dst.alloc(n));
  if (out) MHQ_TRY(dout.alloc(out_cap));
  MHQ_TRY(mhq::launch_write_strings(d->tables, din.p, doff.p, n, dprefix.p, dlead.p, (uint32_t)choice,
                                    out ? dout.p : nullptr, out_cap, dout_off.p, dst.p, s));
  MHQ_TRY(dout_off.get(out_off, n + 1, s));
  MHQ_TRY(hipStreamSynchronize(s));
  if (out) {
    MHQ_TRY(dout.get(out, std::min<uint64_t>(out_off[n], out_cap), s));
    MHQ_TRY(dst.get(status, n, s));
  }
  return hip_rc(hipStreamSynchronize(s));
}

int mhq_read_ints(mhq_ctx *ctx, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos, const uint64_t *limit,
                  const uint8_t *prefix, uint64_t n, int index, uint64_t *value, uint64_t *next, uint8_t *status) {
  Device *d = device(ctx, 0);
  if (!d || (n && (!blk || !pos || !limit || !prefix || !value || !next || !status))) return MHQ_EINVAL;
  for (uint64_t i = 0; i < n; i++)
    if (limit[i] > blk_len) return MHQ_EINVAL;
  std::lock_guard<std::mutex> lock(d->mu);
  MHQ_TRY(hipSetDevice(d->ordinal));
  hipStream_t s = d->stream;
  DevArray<uint8_t> dblk, dprefix, dst;
  DevArray<uint64_t> dpos, dlim, dval, dnext;
  MHQ_TRY(dblk.put(blk, blk_len, s));
  MHQ_TRY(dpos.put(pos, n, s));
  MHQ_TRY(dlim.put(limit, n, s));
  MHQ_TRY(dprefix.put(prefix, n, s));
  MHQ_TRY(dval.alloc(n));
  MHQ_TRY(dnext.alloc(n));
  MHQ_TRY(dst.alloc(n));
  MHQ_TRY(mhq::launch_read_ints(dblk.p, dpos.p, dlim.p, dprefix.p, n, index, dval.p, dnext.p, dst.p, s));
  MHQ_TRY(dval.get(value, n, s));
  MHQ_TRY(dnext.get(next, n, s));
  MHQ_TRY(dst.get(status, n, s));
  return hip_rc(hipStreamSynchronize(s));
}

int mhq_write_ints(mhq_ctx *ctx, const uint64_t *value, const uint8_t *prefix, const uint8_t *lead, uint64_t n,
                   uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint8_t *status) {
  Device *d = device(ctx, 0);
  if (!d || !out_off || (n && (!value || !prefix || !lead || (out && !status)))) return MHQ_EINVAL;
  std::lock_guard<std::mutex> lock(d->mu);
  MHQ_TRY(hipSetDevice(d->ordinal));
  hipStream_t s = d->stream;
  DevArray<uint8_t> dprefix, dlead, dout, dst;
  DevArray<uint64_t> dval, doff;
  MHQ_TRY(dval.put(value, n, s));
  MHQ_TRY(dprefix.put(prefix, n, s));
  MHQ_TRY(dlead.put(lead, n, s));
  MHQ_TRY(doff.alloc(n + 1));
  MHQ_TRY(dst.alloc(n));
  if (out) MHQ_TRY(dout.alloc(out_cap));
  MHQ_TRY(mhq::launch_write_ints(dval.p, dprefix.p, dlead.p, n, out ? dout.p : nullptr, out_cap, doff.p, dst.p, s));
  MHQ_TRY(doff.get(out_off, n + 1, s));
  MHQ_TRY(hipStreamSynchronize(s));
  if (out) {
    MHQ_TRY(dout.get(out, std::min<uint64_t>(out_off[n], out_cap), s));
    MHQ_TRY(dst.get(status, n, s));
  }
  return hip_rc(hipStreamSynchronize(s));
}

int mhq_read_varints(mhq_ctx *ctx, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos, const uint64_t *limit,
                     uint64_t n, uint64_t *value, uint64_t *next, uint8_t *status) {
  Device *d = device(ctx, 0);
  if (!d || (n && (!blk || !pos || !limit || !value || !next || !status))) return MHQ_EINVAL;
  for (uint64_t i = 0; i < n; i++)
    if (limit[i] > blk_len) return MHQ_EINVAL;
  std::lock_guard<std::mutex> lock(d->mu);
  MHQ_TRY(hipSetDevice(d->ordinal));
  hipStream_t s = d->stream;
  DevArray<uint8_t> dblk, dst;
  DevArray<uint64_t> dpos, dlim, dval, dnext;
  MHQ_TRY(dblk.put(blk, blk_len, s));
  MHQ_TRY(dpos.put(pos, n, s));
  MHQ_TRY(dlim.put(limit, n, s));
  MHQ_TRY(dval.alloc(n));
  MHQ_TRY(dnext.alloc(n));
  MHQ_TRY(dst.alloc(n));
  MHQ_TRY(mhq::launch_read_varints(dblk.p, dpos.p, dlim.p, n, dval.p, dnext.p, dst.p, s));
  MHQ_TRY(dval.get(value, n, s));
  MHQ_TRY(dnext.get(next, n, s));
  MHQ_TRY(dst.get(status, n, s));
  return hip_rc(hipStreamSynchronize(s));
}

int mhq_read_frames(mhq_ctx *ctx, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos, const uint64_t *limit,
                    uint64_t n, uint8_t *type, uint64_t *payload_len, uint64_t *payload_pos, uint8_t *status) {
  Device *d = device(ctx, 0);
  if (!d || (n && (!blk || !pos || !limit || !type || !payload_len || !payload_pos || !status))) return MHQ_EINVAL;
  for (uint64_t i = 0; i < n; i++)
    if (limit[i] > blk_len) return MHQ_EINVAL;
  std::lock_guard<std::mutex> lock(d->mu);
  MHQ_TRY(hipSetDevice(d->ordinal));
  hipStream_t s = d->stream;
  DevArray<uint8_t> dblk, dtype, dst;
  DevArray<uint64_t> dpos, dlim, dlen, dppos;
  MHQ_TRY(dblk.put(blk, blk_len, s));
  MHQ_TRY(dpos.put(pos, n, s));
  MHQ_TRY(dlim.put(limit, n, s));
  MHQ_TRY(dtype.alloc(n));
  MHQ_TRY(dlen.alloc(n));
  MHQ_TRY(dppos.alloc(n));
  MHQ_TRY(dst.alloc(n));
  MHQ_TRY(mhq::launch_read_frames(dblk.p, dpos.p, dlim.p, n, dtype.p, dlen.p, dppos.p, dst.p, s));
  MHQ_TRY(dtype.get(type, n, s));
  MHQ_TRY(dlen.get(payload_len, n, s));
  MHQ_TRY(dppos.get(payload_pos, n, s));
  MHQ_TRY(dst.get(status, n, s));
  return hip_rc(hipStreamSynchronize(s));
}

int mhq_write_varints(mhq_ctx *ctx, const uint64_t *value, uint64_t n, uint8_t *out, uint64_t out_cap,
                      uint64_t *out_off, uint8_t *status) {
  Device *d = device(ctx, 0);
  if (!d || !out_off || (n && (!value || (out && !status)))) return MHQ_EINVAL;
  std::lock_guard<std::mutex> lock(d->mu);
  MHQ_TRY(hipSetDevice(d->ordinal));
  hipStream_t s = d->stream;
  DevArray<uint8_t> dout, dst;
  DevArray<uint64_t> dval, doff;
  MHQ_TRY(dval.put(value, n, s));
  MHQ_TRY(doff.alloc(n + 1));
  MHQ_TRY(dst.alloc(n));
  if (out) MHQ_TRY(dout.alloc(out_cap));
  MHQ_TRY(mhq::launch_write_varints(dval.p, n, out ? dout.p : nullptr, out_cap, doff.p, dst.p, s));
  MHQ_TRY(doff.get(out_off, n + 1, s));
  MHQ_TRY(hipStreamSynchronize(s));
  if (out) {
    MHQ_TRY(dout.get(out, std::min<uint64_t>(out_off[n], out_cap), s));
    MHQ_TRY(dst.get(status, n, s));
  }
  return hip_rc(hipStreamSynchronize(s));
}

}  // extern "C"
