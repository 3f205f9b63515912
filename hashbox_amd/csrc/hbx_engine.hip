// hbx_engine.hip — host engine + C-ABI (include/hbxgpu.h) for libhbxgpu.so.
//
// One context = one GPU + one HIP stream + a grown-on-demand workspace.  A
// batch of files runs as five launches on the stream:
//   K1  window-digest scan  grid = tiles (2 MiB of one file each), 1024 thr
//   K2  cut chain           grid = files, 1 wave each (sequential store.go loop)
//   K2c plan                1 workgroup: chunks bucketed by length, longest first
//   K3  block MD5           one 512-thread workgroup per CU, lane per chunk
//   K4  content id          grid = files/64, lane per file
// then one D2H of counts/cuts/ids/content ids into pinned memory.
// Reference seams: hashback/store.go:111-199 (storeFile), pkg/core/client.go:
// 556-560 + block.go:96-111 (StoreData -> HashData).
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hbxgpu.h"
#include "hbx_kernels.hip"

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap && p) return hipSuccess;
    if (p) {
      hipError_t e = hipFree(p);
      if (e != hipSuccess) return e;
      p = nullptr;
      cap = 0;
    }
    size_t want = std::max<size_t>(n, 256);
    want = (want + 4095) & ~size_t(4095);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

struct PinBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap && p) return hipSuccess;
    if (p) {
      (void)hipHostFree(p);
      p = nullptr;
      cap = 0;
    }
    size_t want = std::max<size_t>(n, 4096);
    want = (want + 4095) & ~size_t(4095);
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

struct Pending {
  bool active = false;
  uint64_t n_files = 0;
  uint64_t total_cap = 0;
  uint64_t* cut_ends = nullptr;
  uint8_t* ids = nullptr;
  const uint64_t* out_base = nullptr;
  const uint64_t* caps = nullptr;
  hbx_file_summary* summaries = nullptr;
  std::vector<uint64_t> out_base_copy, caps_copy;
};

}  // namespace

struct hbx_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[5] = {};
  std::mutex mu;
  std::string err;
  uint32_t tile_iters = 64;  // K1 tile = 64 x 64 KiB (measured best: fewer halo primes)
  uint32_t k1_dma = 1;     // K1 lands tiles in LDS by DMA (HBX_K1_DMA=0: register prefetch)
  uint32_t md5_wgs = 256;  // K3 grid: one 512-thread workgroup per CU (set from the device)
  float stage_ms[5] = {0, 0, 0, 0, 0};

  // host-side plan of the current batch
  std::vector<uint64_t> h_slice_base, h_cut_base;
  std::vector<uint2> h_tiles;

  DevBuf d_meta;  // file_off | file_len | slice_base | cut_base | tiles
  DevBuf d_ssum, d_cuts, d_count, d_ids, d_cid, d_ctype, d_work, d_ctl;
  DevBuf d_stage;  // host-input arena
  DevBuf d_msg;    // hbx_block_id message
  PinBuf h_meta, h_res;
  PinBuf h_stage;           // hbx_store_paths: pinned landing buffer for file reads
  hbx_ctx* twin = nullptr;  // hbx_store_paths: second context (double buffering)
  Pending pend;

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
  int hip(hipError_t e, const char* what) {
    if (e == hipSuccess) return HBX_OK;
    err = std::string(what) + ": " + hipGetErrorString(e);
    return HBX_ERR_HIP;
  }
};

#define HBX_TRY(ctx, expr)                                \
  do {                                                    \
    int _rc = (ctx)->hip((expr), #expr);                  \
    if (_rc != HBX_OK) return _rc;                        \
  } while (0)

namespace {

inline uint64_t max_chunks(uint64_t len) { return len / HBX_MIN_BLOCK_SIZE + 1; }

// Layout of the pinned result block after a batch.
struct ResLayout {
  size_t counts, cuts, ids, cid, ctype, total;
};
ResLayout res_layout(uint64_t n_files, uint64_t total_cap) {
  ResLayout r;
  size_t o = 0;
  r.counts = o;
  o += ((n_files * 4 + 255) & ~size_t(255));
  r.cuts = o;
  o += total_cap * 8;
  r.ids = o;
  o += total_cap * 16;
  r.cid = o;
  o += n_files * 16;
  r.ctype = o;
  o += ((n_files * 4 + 255) & ~size_t(255));
  r.total = o;
  return r;
}

// Plan + enqueue one device batch.  Results land in ctx->h_res at the next
// stream sync.
int enqueue_batch(hbx_ctx* c, const void* d_arena, uint64_t n, const uint64_t* offs,
                  const uint64_t* lens, uint64_t* total_cap_out) {
  if (n == 0) {
    *total_cap_out = 0;
    return HBX_OK;
  }
  if (n > 0xFFFFFFFFull) return c->fail(HBX_ERR_ARG, "too many files");
  c->h_slice_base.resize(n);
  c->h_cut_base.resize(n);
  c->h_tiles.clear();
  uint64_t slices = 0, caps = 0;
  const uint64_t tile_bytes = (uint64_t)c->tile_iters * HBX_MIN_BLOCK_SIZE;
  for (uint64_t f = 0; f < n; f++) {
    if (offs[f] % HBX_ARENA_ALIGN) return c->fail(HBX_ERR_ARG, "file offset not 16-byte aligned");
    const uint64_t N = lens[f];
    c->h_slice_base[f] = slices;
    c->h_cut_base[f] = caps;
    const uint64_t cap = max_chunks(N);
    caps += cap;
    if (N > 2ull * HBX_MIN_BLOCK_SIZE) {  // only files with split candidates scan
      slices += (N + kSlice - 1) / kSlice;
      const uint64_t nt = (N + tile_bytes - 1) / tile_bytes;
      if (nt > 0xFFFFFFFFull) return c->fail(HBX_ERR_ARG, "file too large");
      for (uint64_t t = 0; t < nt; t++) c->h_tiles.push_back(make_uint2((uint32_t)f, (uint32_t)t));
    }
  }
  const uint64_t nt = c->h_tiles.size();
  // meta block: off | len | slice_base | cut_base | tiles
  const size_t meta_bytes = n * 8 * 4 + nt * sizeof(uint2);
  HBX_TRY(c, c->h_meta.ensure(meta_bytes));
  HBX_TRY(c, c->d_meta.ensure(meta_bytes));
  uint64_t* hm = c->h_meta.as<uint64_t>();
  std::memcpy(hm, offs, n * 8);
  std::memcpy(hm + n, lens, n * 8);
  std::memcpy(hm + 2 * n, c->h_slice_base.data(), n * 8);
  std::memcpy(hm + 3 * n, c->h_cut_base.data(), n * 8);
  if (nt) std::memcpy(hm + 4 * n, c->h_tiles.data(), nt * sizeof(uint2));

  HBX_TRY(c, c->d_ssum.ensure((slices + 1) * sizeof(uint2)));  // +1: dummy slot
  HBX_TRY(c, c->d_cuts.ensure(caps * 8));
  HBX_TRY(c, c->d_count.ensure(n * 4));
  HBX_TRY(c, c->d_ids.ensure(caps * 16));
  HBX_TRY(c, c->d_work.ensure(caps * 8));
  HBX_TRY(c, c->d_ctl.ensure(64));
  HBX_TRY(c, c->d_cid.ensure(n * 16));
  HBX_TRY(c, c->d_ctype.ensure(n * 4));
  const ResLayout rl = res_layout(n, caps);
  HBX_TRY(c, c->h_res.ensure(rl.total));

  hipStream_t s = c->stream;
  HBX_TRY(c, hipMemcpyAsync(c->d_meta.p, hm, meta_bytes, hipMemcpyHostToDevice, s));
  const uint64_t* d_off = c->d_meta.as<uint64_t>();
  const uint64_t* d_len = d_off + n;
  const uint64_t* d_sb = d_off + 2 * n;
  const uint64_t* d_cb = d_off + 3 * n;
  const uint2* d_tiles = reinterpret_cast<const uint2*>(d_off + 4 * n);
  const uint8_t* arena = static_cast<const uint8_t*>(d_arena);

  HBX_TRY(c, hipEventRecord(c->ev[0], s));
  if (nt) {
    if (c->k1_dma)
      hipLaunchKernelGGL(hbx_k1_digest_scan_dma, dim3((uint32_t)nt), dim3(kK1Threads), 0, s,
                         arena, d_off, d_len, d_sb, d_tiles, c->tile_iters, c->d_ssum.as<uint2>(),
                         slices);
    else
      hipLaunchKernelGGL(hbx_k1_digest_scan, dim3((uint32_t)nt), dim3(kK1Threads), 0, s, arena,
                         d_off, d_len, d_sb, d_tiles, c->tile_iters, c->d_ssum.as<uint2>(),
                         slices);
    HBX_TRY(c, hipGetLastError());
  }
  HBX_TRY(c, hipEventRecord(c->ev[1], s));
  hipLaunchKernelGGL(hbx_k2_cut_chain, dim3((uint32_t)n), dim3(64), 0, s, arena, d_off, d_len,
                     d_sb, c->d_ssum.as<uint2>(), d_cb,
                     c->d_cuts.as<uint64_t>(), c->d_count.as<uint32_t>());
  HBX_TRY(c, hipGetLastError());
  HBX_TRY(c, hipEventRecord(c->ev[2], s));
  hipLaunchKernelGGL(hbx_k2c_plan, dim3(1), dim3(kPlanThreads), 0, s, (uint32_t)n, d_cb,
                     c->d_cuts.as<uint64_t>(), c->d_count.as<uint32_t>(), c->d_work.as<uint2>(),
                     c->d_ctl.as<uint32_t>());
  HBX_TRY(c, hipGetLastError());
  hipLaunchKernelGGL(hbx_k3_block_md5, dim3(c->md5_wgs), dim3(kK3Threads), 0, s, arena, d_off, d_cb,
                     c->d_cuts.as<uint64_t>(), c->d_work.as<uint2>(), c->d_ctl.as<uint32_t>(),
                     c->d_ids.as<uint32_t>());
  HBX_TRY(c, hipGetLastError());
  HBX_TRY(c, hipEventRecord(c->ev[3], s));
  hipLaunchKernelGGL(hbx_k4_content_id, dim3((uint32_t)((n + 63) / 64)), dim3(64), 0, s,
                     (uint32_t)n, d_cb, c->d_count.as<uint32_t>(), c->d_ids.as<uint32_t>(),
                     c->d_cid.as<uint32_t>(), c->d_ctype.as<int32_t>());
  HBX_TRY(c, hipGetLastError());
  HBX_TRY(c, hipEventRecord(c->ev[4], s));

  uint8_t* hr = c->h_res.as<uint8_t>();
  HBX_TRY(c, hipMemcpyAsync(hr + rl.counts, c->d_count.p, n * 4, hipMemcpyDeviceToHost, s));
  HBX_TRY(c, hipMemcpyAsync(hr + rl.cuts, c->d_cuts.p, caps * 8, hipMemcpyDeviceToHost, s));
  HBX_TRY(c, hipMemcpyAsync(hr + rl.ids, c->d_ids.p, caps * 16, hipMemcpyDeviceToHost, s));
  HBX_TRY(c, hipMemcpyAsync(hr + rl.cid, c->d_cid.p, n * 16, hipMemcpyDeviceToHost, s));
  HBX_TRY(c, hipMemcpyAsync(hr + rl.ctype, c->d_ctype.p, n * 4, hipMemcpyDeviceToHost, s));
  *total_cap_out = caps;
  return HBX_OK;
}

// After the stream sync: scatter pinned results into the caller's arrays.
int collect_batch(hbx_ctx* c, uint64_t n, uint64_t total_cap, uint64_t* cut_ends, uint8_t* ids,
                  const uint64_t* out_base, const uint64_t* caps, hbx_file_summary* sums) {
  const ResLayout rl = res_layout(n, total_cap);
  const uint8_t* hr = c->h_res.as<uint8_t>();
  const uint32_t* counts = reinterpret_cast<const uint32_t*>(hr + rl.counts);
  const uint64_t* cuts = reinterpret_cast<const uint64_t*>(hr + rl.cuts);
  const uint8_t* hid = hr + rl.ids;
  const uint8_t* cid = hr + rl.cid;
  const int32_t* ctype = reinterpret_cast<const int32_t*>(hr + rl.ctype);
  int rc = HBX_OK;
  for (uint64_t f = 0; f < n; f++) {
    const uint64_t k = counts[f];
    const uint64_t ib = c->h_cut_base[f];
    if (sums) {
      std::memcpy(sums[f].content_id, cid + 16 * f, 16);
      sums[f].content_type = ctype[f];
      sums[f].n_chunks = (uint32_t)k;
    }
    if (k > caps[f]) {
      rc = c->fail(HBX_ERR_CAPACITY, "output capacity too small for file " + std::to_string(f));
      continue;
    }
    if (cut_ends) std::memcpy(cut_ends + out_base[f], cuts + ib, k * 8);
    if (ids) std::memcpy(ids + 16 * out_base[f], hid + 16 * ib, k * 16);
  }
  float ms = 0.f;
  for (int i = 0; i < 4; i++) {
    if (hipEventElapsedTime(&ms, c->ev[i], c->ev[i + 1]) == hipSuccess) c->stage_ms[i] = ms;
  }
  if (hipEventElapsedTime(&ms, c->ev[0], c->ev[4]) == hipSuccess) c->stage_ms[4] = ms;
  return rc;
}

int run_device_sync(hbx_ctx* c, const void* d_arena, uint64_t n, const uint64_t* offs,
                    const uint64_t* lens, uint64_t* cut_ends, uint8_t* ids,
                    const uint64_t* out_base, const uint64_t* caps, hbx_file_summary* sums) {
  uint64_t total_cap = 0;
  int rc = enqueue_batch(c, d_arena, n, offs, lens, &total_cap);
  if (rc) return rc;
  if (n == 0) return HBX_OK;
  HBX_TRY(c, hipStreamSynchronize(c->stream));
  return collect_batch(c, n, total_cap, cut_ends, ids, out_base, caps, sums);
}

}  // namespace

// ======================================================================
extern "C" {

int hbx_version(void) { return 1; }

int hbx_device_count(int* n) {
  if (!n) return HBX_ERR_ARG;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *n = c;
  return c > 0 ? HBX_OK : HBX_ERR_NODEV;
}

uint64_t hbx_max_chunks(uint64_t len) { return max_chunks(len); }

int hbx_ctx_create(int device, hbx_ctx** out) {
  if (!out) return HBX_ERR_ARG;
  *out = nullptr;
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0) return HBX_ERR_NODEV;
  if (device < 0 || device >= nd) return HBX_ERR_ARG;
  hbx_ctx* c = new hbx_ctx();
  c->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    c->md5_wgs = (uint32_t)prop.multiProcessorCount;
  if (const char* v = std::getenv("HBX_K1_DMA")) c->k1_dma = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("HBX_MD5_WGS")) c->md5_wgs = (uint32_t)std::max(1, std::atoi(v));
  if (const char* v = std::getenv("HBX_TILE_ITERS")) c->tile_iters = (uint32_t)std::min(1024, std::max(1, std::atoi(v)));
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return HBX_ERR_HIP;
  }
  for (auto& e : c->ev) {
    if (hipEventCreate(&e) != hipSuccess) {
      delete c;
      return HBX_ERR_HIP;
    }
  }
  *out = c;
  return HBX_OK;
}

void hbx_ctx_destroy(hbx_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (DevBuf* b : {&c->d_meta, &c->d_ssum, &c->d_cuts, &c->d_count, &c->d_ids,
                    &c->d_cid, &c->d_ctype, &c->d_work, &c->d_ctl, &c->d_stage, &c->d_msg})
    b->release();
  c->h_meta.release();
  c->h_res.release();
  c->h_stage.release();
  if (c->twin) hbx_ctx_destroy(c->twin);
  for (auto& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* hbx_last_error(const hbx_ctx* c) { return c ? c->err.c_str() : "null context"; }

int hbx_set_tile_iters(hbx_ctx* c, uint32_t iters) {
  if (!c || iters == 0 || iters > 1024) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  c->tile_iters = iters;
  return HBX_OK;
}

int hbx_stage_times(hbx_ctx* c, float ms[5]) {
  if (!c || !ms) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  for (int i = 0; i < 5; i++) ms[i] = c->stage_ms[i];
  return HBX_OK;
}

int hbx_chunk_hash_device(hbx_ctx* c, const void* d_arena, uint64_t n, const uint64_t* offs,
                          const uint64_t* lens, uint64_t* cut_ends, uint8_t* ids,
                          const uint64_t* out_base, const uint64_t* caps,
                          hbx_file_summary* sums) {
  if (!c) return HBX_ERR_ARG;
  if (n && (!d_arena || !offs || !lens || !out_base || !caps)) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (c->pend.active) return c->fail(HBX_ERR_STATE, "a submitted batch is still pending");
  HBX_TRY(c, hipSetDevice(c->device));
  return run_device_sync(c, d_arena, n, offs, lens, cut_ends, ids, out_base, caps, sums);
}

int hbx_submit_device(hbx_ctx* c, const void* d_arena, uint64_t n, const uint64_t* offs,
                      const uint64_t* lens, uint64_t* cut_ends, uint8_t* ids,
                      const uint64_t* out_base, const uint64_t* caps, hbx_file_summary* sums) {
  if (!c) return HBX_ERR_ARG;
  if (n && (!d_arena || !offs || !lens || !out_base || !caps)) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (c->pend.active) return c->fail(HBX_ERR_STATE, "a submitted batch is still pending");
  HBX_TRY(c, hipSetDevice(c->device));
  uint64_t total_cap = 0;
  int rc = enqueue_batch(c, d_arena, n, offs, lens, &total_cap);
  if (rc) return rc;
  Pending& p = c->pend;
  p.active = true;
  p.n_files = n;
  p.total_cap = total_cap;
  p.cut_ends = cut_ends;
  p.ids = ids;
  p.summaries = sums;
  p.out_base_copy.assign(out_base, out_base + n);
  p.caps_copy.assign(caps, caps + n);
  return HBX_OK;
}

int hbx_wait(hbx_ctx* c) {
  if (!c) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  Pending& p = c->pend;
  if (!p.active) return HBX_OK;
  p.active = false;
  HBX_TRY(c, hipSetDevice(c->device));
  HBX_TRY(c, hipStreamSynchronize(c->stream));
  if (p.n_files == 0) return HBX_OK;
  return collect_batch(c, p.n_files, p.total_cap, p.cut_ends, p.ids, p.out_base_copy.data(),
                       p.caps_copy.data(), p.summaries);
}

int hbx_chunk_hash_batch(hbx_ctx* c, uint64_t n, const uint8_t* const* datas,
                         const uint64_t* lens, uint64_t* cut_ends, uint8_t* ids,
                         const uint64_t* out_base, const uint64_t* caps,
                         hbx_file_summary* sums) {
  if (!c) return HBX_ERR_ARG;
  if (n && (!datas || !lens || !out_base || !caps)) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (c->pend.active) return c->fail(HBX_ERR_STATE, "a submitted batch is still pending");
  HBX_TRY(c, hipSetDevice(c->device));
  std::vector<uint64_t> offs(n);
  uint64_t total = 0;
  for (uint64_t f = 0; f < n; f++) {
    offs[f] = total;
    total += (lens[f] + 255) & ~uint64_t(255);
  }
  HBX_TRY(c, c->d_stage.ensure(total + 65536));
  uint8_t* arena = c->d_stage.as<uint8_t>();
  for (uint64_t f = 0; f < n; f++) {
    if (lens[f] && !datas[f]) return c->fail(HBX_ERR_ARG, "null file data");
    if (lens[f])
      HBX_TRY(c, hipMemcpyAsync(arena + offs[f], datas[f], lens[f], hipMemcpyHostToDevice,
                                c->stream));
  }
  return run_device_sync(c, arena, n, offs.data(), lens, cut_ends, ids, out_base, caps, sums);
}

int hbx_chunk_hash(hbx_ctx* c, const uint8_t* data, uint64_t len, uint64_t* cut_ends,
                   uint8_t* ids, uint64_t cap, uint64_t* n_chunks) {
  if (!c || (len && !data)) return HBX_ERR_ARG;
  const uint64_t base = 0;
  hbx_file_summary s;
  int rc = hbx_chunk_hash_batch(c, 1, &data, &len, cut_ends, ids, &base, &cap, &s);
  if (n_chunks) *n_chunks = s.n_chunks;
  return rc;
}

int hbx_block_id(hbx_ctx* c, const uint8_t* links, uint32_t n_links, const uint8_t* data,
                 uint64_t len, uint8_t out[16]) {
  if (!c || !out || (n_links && !links) || (len && !data)) return HBX_ERR_ARG;
  if (len > 0xFFFFFFFFull) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HBX_TRY(c, hipSetDevice(c->device));
  const uint64_t n = 8 + 16ull * n_links + len;
  if (n + 16 > 0xFFFFFFFFull) return HBX_ERR_ARG;
  std::vector<uint8_t> msg(n);
  auto be32 = [](uint8_t* b, uint32_t v) {
    b[0] = (uint8_t)(v >> 24);
    b[1] = (uint8_t)(v >> 16);
    b[2] = (uint8_t)(v >> 8);
    b[3] = (uint8_t)v;
  };
  be32(msg.data(), n_links);
  if (n_links) std::memcpy(msg.data() + 4, links, 16ull * n_links);
  be32(msg.data() + 4 + 16ull * n_links, (uint32_t)len);
  if (len) std::memcpy(msg.data() + 8 + 16ull * n_links, data, len);
  HBX_TRY(c, c->d_msg.ensure(n + 16));
  uint8_t* dm = c->d_msg.as<uint8_t>();
  HBX_TRY(c, hipMemcpyAsync(dm + 16, msg.data(), n, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(hbx_k5_md5_raw, dim3(1), dim3(64), 0, c->stream, dm + 16, (uint32_t)n,
                     reinterpret_cast<uint32_t*>(dm));
  HBX_TRY(c, hipGetLastError());
  HBX_TRY(c, hipMemcpyAsync(out, dm, 16, hipMemcpyDeviceToHost, c->stream));
  HBX_TRY(c, hipStreamSynchronize(c->stream));
  return HBX_OK;
}

int hbx_arena_alloc(hbx_ctx* c, uint64_t bytes, void** d_ptr) {
  if (!c || !d_ptr) return HBX_ERR_ARG;
  HBX_TRY(c, hipSetDevice(c->device));
  HBX_TRY(c, hipMalloc(d_ptr, bytes + 65536));
  return HBX_OK;
}

int hbx_arena_free(hbx_ctx* c, void* d_ptr) {
  if (!c) return HBX_ERR_ARG;
  if (!d_ptr) return HBX_OK;
  HBX_TRY(c, hipSetDevice(c->device));
  HBX_TRY(c, hipFree(d_ptr));
  return HBX_OK;
}

int hbx_memcpy_h2d(hbx_ctx* c, void* d, const void* h, uint64_t n) {
  if (!c || (n && (!d || !h))) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HBX_TRY(c, hipSetDevice(c->device));
  HBX_TRY(c, hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, c->stream));
  HBX_TRY(c, hipStreamSynchronize(c->stream));
  return HBX_OK;
}

// ---- files on disk -> pinned -> HBM -> results (BASELINE configs[4]) ----
namespace {

// Read whole files into dst + offs[i] with `threads` threads (files are
// independent).  Returns 0 or HBX_ERR_IO with the offending path in err.
int read_files(uint64_t n, const char* const* paths, const uint64_t* lens, const uint64_t* offs,
               uint8_t* dst, uint32_t threads, std::string& err) {
  std::atomic<uint64_t> next{0};
  std::atomic<int> failed{0};
  std::mutex emu;
  auto worker = [&]() {
    for (;;) {
      const uint64_t i = next.fetch_add(1);
      if (i >= n || failed.load()) return;
      const int fd = ::open(paths[i], O_RDONLY | O_CLOEXEC);
      bool ok = fd >= 0;
      uint64_t got = 0;
      while (ok && got < lens[i]) {
        const ssize_t r = ::pread(fd, dst + offs[i] + got, lens[i] - got, (off_t)got);
        if (r <= 0) ok = false;
        else got += (uint64_t)r;
      }
      if (fd >= 0) ::close(fd);
      if (!ok) {
        failed.store(1);
        std::lock_guard<std::mutex> g(emu);
        err = std::string("cannot read ") + std::to_string(lens[i]) + " bytes of " + paths[i];
        return;
      }
    }
  };
  const uint32_t nt = std::max<uint32_t>(1, std::min<uint64_t>(threads, n));
  std::vector<std::thread> pool;
  for (uint32_t t = 1; t < nt; t++) pool.emplace_back(worker);
  worker();
  for (auto& t : pool) t.join();
  return failed.load() ? HBX_ERR_IO : HBX_OK;
}

}  // namespace

int hbx_store_paths(hbx_ctx* c, uint64_t n, const char* const* paths, const uint64_t* lens,
                    uint64_t* cut_ends, uint8_t* ids, const uint64_t* out_base,
                    const uint64_t* caps, hbx_file_summary* sums, uint32_t io_threads,
                    uint64_t batch_bytes) {
  if (!c) return HBX_ERR_ARG;
  if (n && (!paths || !lens || !out_base || !caps)) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (c->pend.active) return c->fail(HBX_ERR_STATE, "a submitted batch is still pending");
  HBX_TRY(c, hipSetDevice(c->device));
  if (!c->twin) {
    int rc = hbx_ctx_create(c->device, &c->twin);
    if (rc) return c->fail(rc, "cannot create the second context");
    c->twin->tile_iters = c->tile_iters;
    c->twin->md5_wgs = c->md5_wgs;
    c->twin->k1_dma = c->k1_dma;
  }
  if (batch_bytes < (64ull << 20)) batch_bytes = 64ull << 20;
  hbx_ctx* X[2] = {c, c->twin};
  struct Batch {
    uint64_t first = 0, count = 0, total = 0, cap = 0;
    std::vector<uint64_t> offs;
  } B[2];
  auto finish = [&](int s) -> int {  // wait for slot s's batch and scatter its results
    Batch& b = B[s];
    if (!b.count) return HBX_OK;
    HBX_TRY(X[s], hipStreamSynchronize(X[s]->stream));
    int rc = collect_batch(X[s], b.count, b.cap, cut_ends, ids, out_base + b.first,
                           caps + b.first, sums ? sums + b.first : nullptr);
    b.count = 0;
    if (rc) c->err = X[s]->err;
    return rc;
  };
  uint64_t f = 0;
  int slot = 0;
  while (f < n) {
    int rc = finish(slot);  // the slot's buffers are free again
    if (rc) return rc;
    Batch& b = B[slot];
    b.first = f;
    b.offs.clear();
    uint64_t tot = 0;
    while (f < n && (b.offs.empty() || tot + lens[f] <= batch_bytes) && b.offs.size() < 65536) {
      b.offs.push_back(tot);
      tot += (lens[f] + 255) & ~uint64_t(255);
      f++;
    }
    b.count = f - b.first;
    b.total = tot;
    hbx_ctx* x = X[slot];
    HBX_TRY(c, x->h_stage.ensure(tot + 65536));
    HBX_TRY(c, x->d_stage.ensure(tot + 65536));
    rc = read_files(b.count, paths + b.first, lens + b.first, b.offs.data(), x->h_stage.as<uint8_t>(),
                    io_threads, c->err);
    if (rc) {
      b.count = 0;
      (void)finish(slot ^ 1);
      return rc;
    }
    HBX_TRY(c, hipMemcpyAsync(x->d_stage.p, x->h_stage.p, tot, hipMemcpyHostToDevice, x->stream));
    rc = enqueue_batch(x, x->d_stage.p, b.count, b.offs.data(), lens + b.first, &b.cap);
    if (rc) {
      c->err = x->err;
      b.count = 0;
      (void)finish(slot ^ 1);
      return rc;
    }
    slot ^= 1;
  }
  int rc0 = finish(slot);
  int rc1 = finish(slot ^ 1);
  return rc0 ? rc0 : rc1;
}

int hbx_memcpy_h2d_async(hbx_ctx* c, void* d, const void* h, uint64_t n) {
  if (!c || (n && (!d || !h))) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HBX_TRY(c, hipSetDevice(c->device));
  HBX_TRY(c, hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, c->stream));
  return HBX_OK;
}

int hbx_alloc_pinned(uint64_t bytes, void** out) {
  if (!out) return HBX_ERR_ARG;
  return hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault) == hipSuccess ? HBX_OK
                                                                                  : HBX_ERR_HIP;
}

int hbx_free_pinned(void* p) {
  if (!p) return HBX_OK;
  return hipHostFree(p) == hipSuccess ? HBX_OK : HBX_ERR_HIP;
}

}  // extern "C"
