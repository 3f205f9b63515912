// hbx_engine.hip — host engine + C-ABI (include/hbxgpu.h) for libhbxgpu.so.
//
// One context = one GPU + one HIP stream + a grown-on-demand workspace.  A
// batch of files runs as five launches on the stream:
//   K1  window-digest scan  grid = tiles (16 MiB of one file each), 1024 thr
//   K2  cut chain           grid = files, 1 wave each (sequential store.go loop)
//   K2c plan                1 workgroup: chunks bucketed by length, longest first
//   K3  block MD5           one 512-thread workgroup per CU, lane per chunk
//   K4  content id          grid = files/64, lane per file
// then one D2H of counts/cuts/ids/content ids into pinned memory.
// Reference seams: hashback/store.go:111-199 (storeFile), pkg/core/client.go:
// 556-560 + block.go:96-111 (StoreData -> HashData).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <fcntl.h>
#include <unistd.h>

#include <cerrno>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <future>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hbxgpu.h"
#include "hbx_kernels.hip"
#include "hbx_deflate.hip"
#include "hbx_inflate.hip"
#include "hbx_inflate_split.hip"
#include "hbx_formats.h"
#include "hbx_wire.h"

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

// Per-kernel cumulative timing: one event pair per launch, harvested once the
// end event has completed (hbx_stage_totals).  `owned`: the pair came from
// the context's pool (returned there once harvested); a pair of a batch's own
// events (lean marks) stays with the batch.
struct TimedLaunch {
  hipEvent_t a, b;
  int stage;
  bool owned = true;
};

// Layout of a batch's results, the same on the device (d_res) and in the
// pinned host block (h_res), so one copy moves them all.
struct ResLayout {
  size_t counts = 0, cuts = 0, ids = 0, cid = 0, ctype = 0, total = 0;
};
inline size_t al256(size_t x) { return (x + 255) & ~size_t(255); }
ResLayout res_layout(uint64_t n_files, uint64_t total_cap) {
  ResLayout r;
  r.cuts = al256(n_files * 4);
  r.ids = r.cuts + al256(total_cap * 8);
  r.cid = r.ids + al256(total_cap * 16);
  r.ctype = r.cid + al256(n_files * 16);
  r.total = r.ctype + al256(n_files * 4);
  return r;
}

// One submitted batch.  Its device buffers live until its results are
// collected: K3 writes BlockIDs into d_ids across several launches when the
// MD5 stage is time-sliced.
struct Batch {
  uint64_t n = 0, caps = 0;
  std::vector<uint64_t> cut_base;
  DevBuf d_meta, d_res;  // d_res: cut counts | cut ends | ids | content ids | types (rl)
  ResLayout rl;
  uint8_t* res(size_t off) const { return static_cast<uint8_t*>(d_res.p) + off; }
  uint64_t* cuts_d() const { return reinterpret_cast<uint64_t*>(res(rl.cuts)); }
  uint32_t* count_d() const { return reinterpret_cast<uint32_t*>(res(rl.counts)); }
  uint32_t* ids_d() const { return reinterpret_cast<uint32_t*>(res(rl.ids)); }
  DevBuf d_run, d_fresh, d_fcnt;  // the batch's MD5 chains (K2r), their order entries, count
  PinBuf h_meta, h_res;
  uint64_t* cut_ends = nullptr;
  uint8_t* ids = nullptr;
  hbx_file_summary* sums = nullptr;
  std::vector<uint64_t> out_base, capv;
  uint32_t need = 1, done = 0;  // K3 launches its chains need / have had
  bool joined = false;          // its chains are in the carried order lists (a plan took them)
  bool ev3 = false;             // ev[3] recorded (synchronous batches only)
  bool k2_ev5 = false;          // lean marks: K2's end is ev[5] and ev[2] is not recorded
  uint64_t final_launch = 0;    // index of the K3 launch after which it was finalized
  bool finalized = false;
  // a VerifyBlock batch (hbx_verify_submit_device) instead of files
  bool verify = false;
  uint8_t* v_ids = nullptr;
  const uint8_t* v_expect = nullptr;
  uint8_t* v_ok = nullptr;
  uint64_t* v_nbad = nullptr;
  // K1 start | K1 end | K2r end | plan+K3 end (first) | results ready | K2 end (lean marks)
  hipEvent_t ev[6] = {};
  void release() {
    for (DevBuf* d : {&d_meta, &d_res, &d_run, &d_fresh, &d_fcnt}) d->release();
    h_meta.release();
    h_res.release();
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
  }
};

}  // namespace

constexpr uint32_t kK3TimeRing = 4096;  // hbx_ctx::h_k3t slots (2 x u64 each)
constexpr int kDoneRing = 16;         // hbx_ctx::order_free: completion events of the latest K3 launches

struct hbx_ctx {
  int device = 0;
  hipStream_t stream = nullptr;   // scan stream: input copies, K1, K2 (and hbx_block_id)
  hipStream_t cstream = nullptr;  // cut stream: K2 (after its batch's K1 on the scan stream)
  hipStream_t hstream = nullptr;  // hash stream: chain plan, K3
  hipStream_t rstream = nullptr;  // result stream: K4 + result D2H of batches whose chains are done
  hipEvent_t producer = nullptr;  // hbx_after_stream: the caller's stream, waited for on the scan stream
  std::mutex mu;
  std::string err;
  // K1 tile length in 64 KiB iterations; 0 = per batch (k1_tile_iters):
  // about two tiles per CU (four up to 4 GiB), 16..256.  At 8 GiB batches
  // that is 256 (fewer halo primes and, beside K3, fewer, longer K1
  // workgroups: 2,139-2,146 vs 2,088-2,108 GiB/s for 64); a 1 GiB batch gets
  // 16 so that its K1 spreads evenly over the CUs K3 leaves
  uint32_t tile_iters = 0;
  uint32_t join_lag = 1;      // hbx_set_join_lag
  // where and when K2c plans run follows from the join lag (plan_mode_of)
  bool preplanned = false;    // the plan of launch `launches` is enqueued (mode 2)
  std::vector<Batch*> pre_nb; // the batches whose chains that plan adds
  // K3 period (hbx_set_k3_period): one K3 launch every `k3_period` submits,
  // with `k3_period` x the slice per chain, joining every batch old enough:
  // the launch's fixed start-up and tail are paid once per period (small
  // per-GPU batches, the N = 8 share of configs[2]).  k3_tick counts submits.
  uint32_t k3_period = 1;
  uint64_t k3_tick = 0;
  uint32_t k4_window = 1024;  // K4's LDS window of ids (HBX_K4_WINDOW, 1..1024: tests)
  int k2_own = -1;            // ensure_cut_stream: -1 = by join lag (HBX_K2_STREAM for A/B)
  uint32_t md5_wgs = 256;     // K3 grid: one 256-thread workgroup per CU (set from the device)
  // K3P: a producer wave per MD5 wave (HBX_K3_PROD=0 for the self-staging K3,
  // A/B): 1,435 vs 1,586 cycles per block inside the bench schedule, +1.7 %
  // (200 steps) and +2.9 % at 8 files per GPU (profiles/r05f)
  uint32_t k3_prod = 1;
  // K3P producer register sets in flight: 3 (a stage more of memory latency
  // hidden) 2,297-2,318 vs 2,286-2,308 GiB/s in three alternating pairs at 64
  // files, equal at 8 (profiles/r05af); HBX_K3_PSETS=2 for A/B
  uint32_t k3_psets = 3;
  uint32_t k3_spin = 0;
  // full-slice chains ordered by data address in plan_addr granules of
  // 2^plan_addr_shift bytes (plan_bin; HBX_PLAN_ADDR=0..512, 0 = by count
  // only as before round 6; HBX_PLAN_ADDR_SHIFT=20..40)
  uint32_t plan_addr = 512, plan_addr_shift = 29;
  // K1 launched with its batch's ev[0]/ev[1] as hipExtLaunchKernel start/stop
  // events instead of marker packets around it (HBX_K1_EXT=0: markers)
  uint32_t k1_ext = 1;
  uint32_t k1_dma4 = 1;  // K1's four LDS-DMA pieces in one statement (HBX_K1_DMA4=0: one per piece)
  // K1's first two DMA iterations issued before the halo's loads (HBX_K1_EARLY=0:
  // after the prime); one memory round trip per tile fewer in principle,
  // neutral in measurement (64 files 2,328/2,329 vs 2,337/2,351, 8 files
  // 2,075/2,082 vs 2,041/2,062 GiB/s, profiles/r06u)
  uint32_t k1_early = 1;
  // at join lag 2, preplan on the cut stream (mode 3; HBX_PLAN_CUT=0: mode 1,
  // the plan on the hash stream): +2.7 % with K3P (profiles/r05e)
  // 2 (default): at lag 3 and 4 too, off the scan loop (8 files per GPU, K3
  // period 4: 2,075-2,079 vs 2,031-2,049 GiB/s, profiles/r05l); 1: lag 2 only
  uint32_t plan_cut = 2;
  // the batch meta reaches the device by hbx_meta_fetch, a kernel on the scan
  // stream, instead of an SDMA copy (HBX_META_KERNEL=0 for A/B)
  uint32_t meta_kernel = 1;
  // round 6: the meta copy inside the K1 gate kernel (hbx_k1_gate_meta), one
  // scan-stream kernel fewer per step (HBX_GATE_META=0: separate kernels)
  uint32_t gate_meta = 1;
  // a finished batch's results reach the host by hbx_result_push, a kernel
  // on the result stream, instead of an SDMA copy (HBX_D2H_KERNEL=0 for A/B):
  // the copy call held the host ~7 ms once per ~16 submits after a drain
  // (profiles/r05az: 8-file 20-step window 1,395 -> 1,994-2,033 GiB/s)
  uint32_t d2h_kernel = 64;  // workgroups (0 = SDMA copy)
  // K1's LDS image transposed per 1 KiB: its per-lane reads become
  // conflict-free (SQ_LDS_BANK_CONFLICT 1.0e8 -> 0 per launch), K1 beside K3
  // 3.26 -> 3.19 ms per 8 GiB (profiles/r05ab); HBX_K1_SWZ=0 for the old image
  uint32_t k1_swz = 1;
  // K3Q: items per group (parts of each slice, handed out through a queue;
  // 0 = off, K3P's static groups; HBX_K3_ITEMS for A/B)
  uint32_t k3_items = 0;
  PinBuf h_err;  // K3Q: set by a wave that gave up waiting for an item (never expected)
  uint32_t md5_slice = 16384; // K3 time slice: full MD5 blocks per chain per launch (0 = unlimited)
  // K1 gate (hbx_k1_gate): a batch's K1 waits until every workgroup of the K3
  // launch of the same submit has been dispatched.  k3_started counts K3
  // workgroups on the device; k3_dispatched is the host's running total.
  uint32_t k1_gate = 1;
  // Lean marks (HBX_LEAN_MARKS=0 for A/B): every event record or zero-fill
  // between two kernels of one stream costs ~5 us of dispatch, and the scan
  // stream's gate -> K1 -> K2 -> K2r -> plan is one of the step's two
  // equal-length loops.  With them K1 and K2 are timed by the
  // batch's own ev[0] | ev[1] | ev[5], K2 zeroes K2r's counter, the plan's
  // timing end event is what K3 waits on, and the plan bins are zeroed
  // after each plan (off the loop) instead of before it.
  uint32_t lean_marks = 1;  // 0 off (the old schedule, A/B), 1 on
  hipStream_t plan_zeroed_on = nullptr;  // stream whose last op leaves d_plan zeroed (lean)
  TimedLaunch plan_timer[3];             // lean: the plan's timing pair, queued once K3 waits on it
  bool plan_timer_set[3] = {false, false, false};
  hipEvent_t plan_wait[3] = {nullptr, nullptr, nullptr};  // what K3 of launch j%3 waits on
  // lean: hbx_input_after_oldest's wait (for K3 launch input_wait_L), enqueued
  // on the scan stream only just before the next thing that could touch the
  // old input (flush_input_wait), i.e. after the plan instead of before it
  bool input_wait_pending = false;
  uint64_t input_wait_L = 0;
  // the launch the latest hbx_input_after_oldest ordered input behind
  // (hbx_input_fence hands it to a caller's stream); unset once known complete
  bool input_fence_set = false;
  uint64_t input_fence_L = 0;
  DevBuf d_gate;
  uint32_t k3_dispatched = 0;
  // K3 launch times measured on the device (no timing events on the hash
  // stream, which carries only K3 and its completion event): K3's first
  // workgroup and its last wave stamp s_memrealtime into slot (launch %
  // kK3TimeRing) of this pinned ring; tickets from d_gate[0] (workgroups
  // started) and d_gate[1] (waves ended).  Harvested once a launch is known
  // complete (k3_done_upto: launches [0, k3_done_upto) are).
  PinBuf h_k3t;
  PinBuf h_probe;  // hbx_set_k3_probe: per-wave times of the latest K3 launch (hbx_k3_wave_times)
  uint32_t k3_waves = 0;
  std::deque<uint64_t> k3_open;
  uint64_t k3_done_upto = 0;
  float stage_ms[5] = {0, 0, 0, 0, 0};

  // host-side plan scratch
  std::vector<uint64_t> h_slice_base;
  std::vector<uint4> h_tiles;

  // K1 -> K2 slice summaries, two slots used by alternate batches: K1 of
  // batch i+1 (scan stream) overlaps K2 of batch i (cut stream)
  DevBuf d_ssum[2];
  int ssum_slot = 0;
  hipEvent_t ssum_free[2] = {nullptr, nullptr};  // recorded after the K2 that last read the slot
  bool ssum_used[2] = {false, false};
  // K3 launch orders (triple-buffered by launch index % 3): plan j (scan
  // stream) writes order[j%3] from order[(j-1)%3]; K3 j (hash stream) reads it
  DevBuf d_order[3], d_octl[3], d_q[3];  // (+ K3Q's item queue per slot)
  hipEvent_t plan_done[3] = {nullptr, nullptr, nullptr};   // plan j%3 written
  // completion of K3 launch L: order_free[L % kDoneRing] (recorded again by
  // launch L + kDoneRing).  The plan of launch j waits for launch j - 3, the
  // last reader of its order slot; hbx_input_after_oldest for the launch that
  // finished the oldest batch, which with a K3 period or a long lead is
  // several launches back (with 3 events it fell back to the newest launch,
  // serializing the next K1 behind the running K3: 8 files per GPU at K3
  // period 8 and lead 11, 1,579 vs 2,079 GiB/s, profiles/r05n)
  hipEvent_t order_free[kDoneRing] = {};
  uint64_t launches = 0;    // K3 launches planned so far
  uint32_t last_budget = 0; // budget of the last planned launch
  DevBuf d_stage;           // host-input arena
  DevBuf d_msg;             // hbx_block_id message
  DevBuf d_plan;            // chain planner: global bin counts + cursors
  DevBuf d_vdesc, d_vlinks, d_vout, d_vexp, d_zeros;  // hbx_verify_blocks*
  DevBuf d_zblk, d_zinfo, d_zoff, d_zlen, d_zout, d_zimg;  // hbx_deflate_blocks*
  DevBuf d_idesc, d_ires;                                  // hbx_inflate_blocks_device
  DevBuf d_sreg, d_sstart, d_sres, d_sscratch, d_smeta;    // its split path (K8s)
  uint64_t k8_split_streams = 0, k8_split_fallbacks = 0;   // (hbx_knobs: how often the split path resolved)
  // SDMA engines warmed at context creation (warm_sdma_engines): H2D and D2H
  // engine masks, and the milliseconds this context spent on it (0 once the
  // process has done it for the device)
  uint32_t sdma_h2d = 0, sdma_d2h = 0;
  double sdma_warm_ms = 0.0;
  // hbx_host_call_max: the longest host time of one H2D copy call and of one
  // batch submit since the last reset (hbx_memcpy_h2d_async, the disk path's
  // copies, submit_batch), ms
  double max_copy_ms = 0.0, max_submit_ms = 0.0;
  uint32_t sdma_warm = 1;
  PinBuf h_read[2];         // hbx_store_paths: pinned landing slots for file reads
  PinBuf h_zstage;          // hbx_store_paths_z: compressed streams of one batch (synchronous form)
  // hbx_store_paths_z: compression stages in flight, each on its own stream
  static constexpr int kZStages = 2;  // three measured slower (16.1 vs 21.8 GiB/s, profiles/r02i_zpipe)
  struct ZStage {
    DevBuf blk, info, off, len, img, out;
    PinBuf desc, lens, stage;
    hipEvent_t done = nullptr;
    hipStream_t stream = nullptr;  // one per stage: one job's K7 overlaps another's copy-back
  } zs[kZStages];
  hipEvent_t h2d_done[2] = {nullptr, nullptr};  // slot's H2D copy has completed
  std::vector<DevBuf> d_ring;  // hbx_store_paths: device arenas of the batches in flight
  double io_s[3] = {0, 0, 0};  // hbx_store_paths: reading files | waiting for an arena | waiting for a copy

  std::deque<Batch*> pending;  // submitted, not yet collected (FIFO)
  std::vector<Batch*> pool;
  // A HIP error after a batch's device work was enqueued leaves chains of it
  // in the carried order lists: the context refuses further pipelined work
  // (HBX_ERR_STATE) and the batch's buffers are parked here, never reused,
  // until hbx_ctx_destroy.
  bool broken = false;
  std::vector<Batch*> parked;
  // Batches whose chains are cut (K2r enqueued) but not yet in a plan, oldest
  // first: a batch joins the K3 launch issued `join_lag` submits after its
  // own (or a wait's drain), so K3 launch j never waits for batch j's own
  // scan and the scan side runs join_lag steps ahead of the hash stream.
  std::deque<Batch*> unjoined;
  std::vector<TimedLaunch> open_t;
  std::vector<hipEvent_t> ev_pool;
  double tot_ms[5] = {0, 0, 0, 0, 0};
  uint64_t tot_n[5] = {0, 0, 0, 0, 0};

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
  int hip(hipError_t e, const char* what) {
    if (e == hipSuccess) return HBX_OK;
    err = std::string(what) + ": " + hipGetErrorString(e);
    return HBX_ERR_HIP;
  }
  hipEvent_t event() {
    if (!ev_pool.empty()) {
      hipEvent_t e = ev_pool.back();
      ev_pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    return hipEventCreate(&e) == hipSuccess ? e : nullptr;
  }
};

#define HBX_TRY(ctx, expr)                                \
  do {                                                    \
    int _rc = (ctx)->hip((expr), #expr);                  \
    if (_rc != HBX_OK) return _rc;                        \
  } while (0)

namespace {

inline uint64_t max_chunks(uint64_t len) { return len / HBX_MIN_BLOCK_SIZE + 1; }

// Grow a buffer the streams may still be using: drain both streams first.  A
// drain stalls the pipeline, so growth is geometric (and hbx_reserve sizes
// everything up front for a known workload).
int ensure_shared(hbx_ctx* c, DevBuf& b, size_t n) {
  if (n <= b.cap && b.p) return HBX_OK;
  HBX_TRY(c, hipStreamSynchronize(c->stream));
  HBX_TRY(c, hipStreamSynchronize(c->cstream));
  HBX_TRY(c, hipStreamSynchronize(c->hstream));
  HBX_TRY(c, hipStreamSynchronize(c->rstream));
  HBX_TRY(c, b.ensure(b.p ? std::max(n, b.cap + b.cap / 2) : n));
  return HBX_OK;
}

// Bracket one launch with an event pair for hbx_stage_totals.
struct StageTimer {
  hbx_ctx* c;
  hipStream_t s;
  TimedLaunch t;
  // on = false: a no-op (the caller times the launch with events it records anyway)
  StageTimer(hbx_ctx* ctx, hipStream_t st, int stage, bool on = true) : c(ctx), s(st) {
    t.stage = stage;
    t.a = on ? c->event() : nullptr;
    t.b = on ? c->event() : nullptr;
    if (t.a) (void)hipEventRecord(t.a, s);
  }
  ~StageTimer() {
    if (!t.a && !t.b) return;
    if (t.a && t.b && hipEventRecord(t.b, s) == hipSuccess) {
      c->open_t.push_back(t);
    } else {
      if (t.a) c->ev_pool.push_back(t.a);
      if (t.b) c->ev_pool.push_back(t.b);
    }
  }
};

// Timed launches of one stage run on one stream, so they complete in order:
// once one is still running, the later ones of its stage are not queried (a
// host far ahead of the device keeps many open, and each query costs µs).
void harvest_timings(hbx_ctx* c) {
  size_t keep = 0;
  bool open[5] = {false, false, false, false, false};
  for (size_t i = 0; i < c->open_t.size(); i++) {
    TimedLaunch& t = c->open_t[i];
    float ms = 0.f;
    bool done = false;
    if (!open[t.stage]) {
      done = hipEventQuery(t.b) == hipSuccess && hipEventElapsedTime(&ms, t.a, t.b) == hipSuccess;
      open[t.stage] = !done;
    }
    if (done) {
      c->tot_ms[t.stage] += ms;
      c->tot_n[t.stage] += 1;
      if (t.owned) {
        c->ev_pool.push_back(t.a);
        c->ev_pool.push_back(t.b);
      }
    } else {
      c->open_t[keep++] = t;
    }
  }
  c->open_t.resize(keep);
}


// Add the device-measured K3 launches known complete to the totals.
void harvest_k3(hbx_ctx* c) {
  while (!c->k3_open.empty() && c->k3_open.front() < c->k3_done_upto) {
    const volatile uint64_t* t = c->h_k3t.as<uint64_t>() + 2 * (c->k3_open.front() % kK3TimeRing);
    const uint64_t a = t[0], e = t[1];
    if (a && e >= a) {
      c->tot_ms[3] += (double)(e - a) * 1e-5;  // s_memrealtime: 100 MHz
      c->tot_n[3] += 1;
    }
    c->k3_open.pop_front();
  }
}

Batch* acquire_batch(hbx_ctx* c) {
  Batch* b;
  if (!c->pool.empty()) {
    b = c->pool.back();
    c->pool.pop_back();
  } else {
    b = new Batch();
    for (auto& e : b->ev) {
      if (hipEventCreate(&e) != hipSuccess) {
        b->release();
        delete b;
        return nullptr;
      }
    }
  }
  b->n = b->caps = 0;
  b->need = 1;
  b->done = 0;
  b->rl = ResLayout{};  // a verify batch keeps its ids at offset 0 of d_res
  b->joined = false;
  b->ev3 = false;
  b->k2_ev5 = false;
  b->final_launch = 0;
  b->finalized = false;
  b->cut_ends = nullptr;
  b->ids = nullptr;
  b->sums = nullptr;
  b->verify = false;
  b->v_ids = nullptr;
  b->v_expect = nullptr;
  b->v_ok = nullptr;
  b->v_nbad = nullptr;
  return b;
}

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

// HBX_TRACE_SLOW_SUBMIT=<ms>: a submit slower than that prints where its host
// time went (diagnostics for one-off host stalls; off by default).
struct SlowSubmit {
  double limit_ms = -1.0;
  double fin[3] = {0, 0, 0};  // finalize: K4 (+ its timing events), D2H copy, completion record
  std::chrono::steady_clock::time_point t[12];
  SlowSubmit() {
    if (const char* v = std::getenv("HBX_TRACE_SLOW_SUBMIT")) limit_ms = std::atof(v);
  }
  void mark(int i) {
    if (limit_ms >= 0) t[i] = std::chrono::steady_clock::now();
  }
  void report(uint64_t launches) {
    if (limit_ms < 0) return;
    auto ms = [&](int a, int b) { return std::chrono::duration<double, std::milli>(t[b] - t[a]).count(); };
    if (ms(0, 5) < limit_ms) return;
    std::fprintf(stderr, "hbx slow submit (launch %llu): %.3f ms = setup %.3f, buffers %.3f, md5_step %.3f, preplan %.3f, scan %.3f"
                 " | md5_launch: entry %.3f, k3 launch %.3f, record %.3f, finalize %.3f\n",
                 (unsigned long long)launches, ms(0, 5), ms(0, 1), ms(1, 2), ms(2, 3), ms(3, 4), ms(4, 5),
                 ms(2, 6), ms(6, 7), ms(7, 8), ms(8, 9));
    std::fprintf(stderr, "  finalize: k4 %.3f, d2h %.3f, record %.3f\n", fin[0], fin[1], fin[2]);
  }
  void clear() {
    if (limit_ms < 0) return;
    for (int i = 6; i < 10; i++) t[i] = t[0];
    fin[0] = fin[1] = fin[2] = 0;
  }
  // one host call outside submit (e.g. the H2D copy call), reported alone
  void call(const char* what, std::chrono::steady_clock::time_point a, uint64_t launches) {
    if (limit_ms < 0) return;
    const double d = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
    if (d >= limit_ms)
      std::fprintf(stderr, "hbx slow call (launch %llu): %s %.3f ms\n", (unsigned long long)launches, what, d);
  }
  void lap(int k, std::chrono::steady_clock::time_point& a) {
    if (limit_ms < 0) return;
    const auto b = std::chrono::steady_clock::now();
    fin[k] += std::chrono::duration<double, std::milli>(b - a).count();
    a = b;
  }
};
// Per thread (advisor r05): a context's calls are serialised by its own lock
// only, so contexts submitting from different threads must not share it; two
// contexts on one thread never overlap.
static thread_local SlowSubmit g_slow;

// K4 + D2H of one batch whose chains are all hashed, on the result stream
// (after the finalizing K3's completion event), so the hash stream goes straight on with the next plan
// and K3 launch.
int finalize_batch(hbx_ctx* c, Batch* b) {
  hipStream_t s = c->rstream;
  b->finalized = true;
  if (b->verify) {
    if (b->n) HBX_TRY(c, hipMemcpyAsync(b->h_res.p, b->d_res.p, b->n * 16, hipMemcpyDeviceToHost, s));
    HBX_TRY(c, hipEventRecord(b->ev[4], s));
    return HBX_OK;
  }
  auto lap = std::chrono::steady_clock::now();
  if (b->n) {
    const uint64_t n = b->n;
    const uint64_t* d_cb = b->d_meta.as<uint64_t>() + 3 * n;
    {
      StageTimer t(c, s, 4);
      hipLaunchKernelGGL(hbx_k4_content_id, dim3((uint32_t)n), dim3(64), 0, s,
                         (uint32_t)n, d_cb, b->count_d(), b->ids_d(), reinterpret_cast<uint32_t*>(b->res(b->rl.cid)),
                         reinterpret_cast<int32_t*>(b->res(b->rl.ctype)), c->k4_window);
    }
    HBX_TRY(c, hipGetLastError());
    g_slow.lap(0, lap);
    // one copy for every result (5 copies before: each a dispatch on this stream)
    if (c->d2h_kernel && b->rl.total % 16 == 0) {
      const uint64_t n16 = b->rl.total / 16;
      hipLaunchKernelGGL(hbx_result_push, dim3((uint32_t)std::min<uint64_t>(c->d2h_kernel, (n16 + 255) / 256)),
                         dim3(256), 0, s, b->d_res.as<uint4>(), static_cast<uint4*>(b->h_res.p), n16);
      HBX_TRY(c, hipGetLastError());
    } else {
      HBX_TRY(c, hipMemcpyAsync(b->h_res.p, b->d_res.p, b->rl.total, hipMemcpyDeviceToHost, s));
    }
    g_slow.lap(1, lap);
  }
  HBX_TRY(c, hipEventRecord(b->ev[4], s));
  g_slow.lap(2, lap);
  return HBX_OK;
}

// One MD5 launch: plan (carried chains + the new batch's chunks, if any) and
// K3 with `budget` blocks per chain.  Afterwards every pending batch has had
// one more launch; those whose chains are now guaranteed complete are
// finalized.  A budget of kBudgetAll completes every chain in flight.
// Plan launch j = c->launches on the scan stream: order[j%3] from
// order[(j-1)%3] (advanced by the budget of launch j-1) plus the fresh chains
// of batch nb (if any).  Needs no result of any K3 launch.
int ensure_plan_buffers(hbx_ctx* c, uint64_t extra);

// Where and when plans run (the plan of launch j+1 adds batch j+1-lag).
// * lag 1, mode 0: submit j+1 enqueues it on the scan stream, after batch j's
//   K1 (and K2), whose chains it adds.
// * lag 2, mode 1: the batch was cut a step earlier, so the plan can go on the
//   hash stream between K3 j and K3 j+1, off the scan stream (which then
//   carries only the K1 gate and K1).  Costs ~0.06 ms of dispatch gaps per
//   step on the hash stream.
// * lag >= 3, mode 2 (preplan): submit j enqueues it on the scan stream right
//   after launching K3 j and BEFORE batch j's K1; the batch it adds (j-2 or
//   older) was cut during the previous step, so the plan never waits for a K2
//   and the hash stream carries nothing but K3 launches.  At lag 2 the same
//   schedule would make K1 j wait for K2 of batch j-1 (measured 1,575 GiB/s at
//   8 files per GPU, vs 1,890 for mode 1).
// * lag 2, mode 3 (preplan on the cut stream, c->plan_cut): the same preplan
//   as mode 2, but on the cut stream, right behind batch j-1's K2 and K2r
//   (whose chains it adds) and before batch j's K2: neither the scan stream
//   nor the hash stream waits for it, and the hash stream carries nothing but
//   K3 launches.
// The blocks per chain of one K3 launch for a per-submit slice `budget`.
uint32_t launch_budget(const hbx_ctx* c, uint32_t budget) {
  if (budget == kBudgetAll || c->k3_period <= 1) return budget;
  return (uint32_t)std::min<uint64_t>((uint64_t)budget * c->k3_period, kBudgetAll - 1);
}

int plan_mode_of(const hbx_ctx* c) {
  if ((c->join_lag == 2 ? c->plan_cut : c->plan_cut > 1 && c->join_lag > 2) && c->cstream != c->stream) return 3;
  return c->join_lag >= 3 ? 2 : c->join_lag == 2 ? 1 : 0;
}
hipStream_t plan_stream(const hbx_ctx* c) {
  const int m = plan_mode_of(c);
  return m == 1 ? c->hstream : m == 3 ? c->cstream : c->stream;
}

// K2 + K2r get a stream of their own once the join lag allows it (or
// HBX_K2_STREAM=1): K1 of the next batch then no longer queues behind this
// batch's K2 (at 8 files per GPU, 1,578 -> 1,825 GiB/s).  At lag 1 the plan
// needs K2r right away, and a fourth stream of ours shares one of the
// GPU_MAX_HW_QUEUES = 4 hardware queues (measured +0.2 ms hash-stream gap),
// so K2 stays on the scan stream.  Created once; never dropped.
int ensure_cut_stream(hbx_ctx* c) {
  const bool want = c->k2_own < 0 ? c->join_lag >= 2 : c->k2_own > 0;
  if (!want || c->cstream != c->stream || c->hstream == c->stream) return HBX_OK;
  hipStream_t s = nullptr;
  HBX_TRY(c, hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  c->cstream = s;
  return HBX_OK;
}

// Enqueue a deferred hbx_input_after_oldest wait on the scan stream (nothing
// once the host has seen that launch complete).  Called before anything that
// may read or write a caller's input on the scan stream, and before any K3
// launch could record the launch's completion slot again.
int flush_input_wait(hbx_ctx* c) {
  if (!c->input_wait_pending) return HBX_OK;
  c->input_wait_pending = false;
  hipEvent_t e = c->order_free[c->input_wait_L % kDoneRing];
  if (hipEventQuery(e) == hipSuccess) return HBX_OK;
  HBX_TRY(c, hipStreamWaitEvent(c->stream, e, 0));
  return HBX_OK;
}

int plan_launch(hbx_ctx* c, const std::vector<Batch*>& nbs, uint32_t budget) {
  hipStream_t s = plan_stream(c);
  const int slot = (int)(c->launches % 3), ps = (int)((c->launches + 2) % 3);
  int rc = ensure_plan_buffers(c, 0);  // nb (if any) is already in pending
  if (rc) return rc;
  // the K3 launch that read this slot three launches ago must be done (lean:
  // no wait enqueued once the host has seen it complete, the usual case)
  if (c->launches >= 3 && c->hstream != s) {
    hipEvent_t e = c->order_free[(c->launches - 3) % kDoneRing];
    if (!(c->lean_marks && hipEventQuery(e) == hipSuccess)) HBX_TRY(c, hipStreamWaitEvent(s, e, 0));
  }
  // carried chains exist only while an older batch is unfinalized (a batch
  // is finalized once every chain of it is hashed); without one the previous
  // list is not read at all (hbx_reserve may have reallocated it)
  bool has_prev = false;
  for (Batch* b : c->pending)
    if (b->joined && !b->finalized && std::find(nbs.begin(), nbs.end(), b) == nbs.end()) has_prev = true;
  has_prev = has_prev && c->launches > 0;
  FreshSet fs{};
  for (Batch* nb : nbs) {
    if (!nb->n) continue;
    fs.f[fs.k] = nb->d_fresh.as<OrderEntry>();
    fs.n[fs.k] = nb->d_fcnt.as<uint32_t>();
    fs.k++;
    // the joining batch's chains come from K2r (cut stream) or K6p (scan stream)
    if (!(s == c->stream && c->cstream == s)) HBX_TRY(c, hipStreamWaitEvent(s, nb->ev[2], 0));
  }
  // the plan stream changed (hbx_set_join_lag): the trailing bin fill queued on
  // the old one must not land inside this plan
  if (c->plan_zeroed_on && c->plan_zeroed_on != s) {
    HBX_TRY(c, hipStreamSynchronize(c->plan_zeroed_on));
    c->plan_zeroed_on = nullptr;
  }
  if (c->lean_marks) {
    TimedLaunch t;
    t.stage = 2;
    t.a = c->event();
    t.b = c->event();
    if (t.a && t.b) {
      HBX_TRY(c, hipEventRecord(t.a, s));
      if (c->plan_zeroed_on != s) HBX_TRY(c, hipMemsetAsync(c->d_plan.p, 0, 2 * kPlanBins * sizeof(uint32_t), s));
      for (uint32_t phase = 0; phase < 2; phase++)
        hipLaunchKernelGGL(hbx_k2c_plan, dim3(kPlanGroups), dim3(kPlanThreads), 0, s,
                           has_prev ? c->d_order[ps].as<OrderEntry>() : nullptr,
                           has_prev ? c->d_octl[ps].as<uint32_t>() : nullptr, c->last_budget,
                           fs, budget, c->d_order[slot].as<OrderEntry>(), c->d_octl[slot].as<uint32_t>(),
                           c->d_plan.as<uint32_t>(), phase | (c->plan_addr << 8) | (c->plan_addr_shift << 24));
      HBX_TRY(c, hipGetLastError());
      HBX_TRY(c, hipEventRecord(t.b, s));
      // K3 waits on the timing end itself; the pair is queued for harvest
      // only once that wait is enqueued (md5_launch), so the pool cannot hand
      // t.b out again before
      if (c->plan_timer_set[slot]) c->open_t.push_back(c->plan_timer[slot]);  // (not reached: K3 took it)
      c->plan_timer[slot] = t;
      c->plan_timer_set[slot] = true;
      c->plan_wait[slot] = t.b;
      // the bins for the next plan, while K3 is being dispatched
      c->plan_zeroed_on = nullptr;
      HBX_TRY(c, hipMemsetAsync(c->d_plan.p, 0, 2 * kPlanBins * sizeof(uint32_t), s));
      c->plan_zeroed_on = s;
      return flush_input_wait(c);
    }
    if (t.a) c->ev_pool.push_back(t.a);
    if (t.b) c->ev_pool.push_back(t.b);
  }
  c->plan_zeroed_on = nullptr;
  {
    StageTimer t(c, s, 2);
    HBX_TRY(c, hipMemsetAsync(c->d_plan.p, 0, 2 * kPlanBins * sizeof(uint32_t), s));
    for (uint32_t phase = 0; phase < 2; phase++)
      hipLaunchKernelGGL(hbx_k2c_plan, dim3(kPlanGroups), dim3(kPlanThreads), 0, s,
                         has_prev ? c->d_order[ps].as<OrderEntry>() : nullptr,
                         has_prev ? c->d_octl[ps].as<uint32_t>() : nullptr, c->last_budget,
                         fs, budget, c->d_order[slot].as<OrderEntry>(), c->d_octl[slot].as<uint32_t>(),
                         c->d_plan.as<uint32_t>(), phase | (c->plan_addr << 8) | (c->plan_addr_shift << 24));
  }
  HBX_TRY(c, hipGetLastError());
  HBX_TRY(c, hipEventRecord(c->plan_done[slot], s));
  c->plan_wait[slot] = c->plan_done[slot];
  return flush_input_wait(c);
}

// One MD5 launch (planned by plan_launch just before): K3 with `budget`
// blocks per chain.  Afterwards every pending batch has had one more launch;
// those whose chains are now guaranteed complete are finalized.  A budget of
// kBudgetAll completes every chain in flight.
int md5_launch(hbx_ctx* c, const std::vector<Batch*>& nbs, uint32_t budget) {
  if (int frc = flush_input_wait(c)) return frc;  // (a preplanned launch comes without a plan_launch)
  hipStream_t s = c->hstream;
  const int slot = (int)(c->launches % 3);
  if (s != plan_stream(c)) HBX_TRY(c, hipStreamWaitEvent(s, c->plan_wait[slot], 0));
  if (c->plan_timer_set[slot]) {  // lean marks: the wait is enqueued, the pair may be harvested
    c->open_t.push_back(c->plan_timer[slot]);
    c->plan_timer_set[slot] = false;
  }
  // the device-timing slot of this launch (its previous user, kK3TimeRing
  // launches back, must have been harvested)
  const uint64_t L = c->launches;
  if (!c->k3_open.empty() && c->k3_open.front() + kK3TimeRing <= L) {
    HBX_TRY(c, hipStreamSynchronize(s));
    c->k3_done_upto = L;
    harvest_k3(c);
  }
  uint64_t* tslot = nullptr;
  if (c->h_k3t.p) {
    tslot = c->h_k3t.as<uint64_t>() + 2 * (L % kK3TimeRing);
    tslot[0] = tslot[1] = 0;
    c->k3_open.push_back(L);
  }
  const uint32_t waves = c->md5_wgs * (kK3Threads / 64);
  g_slow.mark(6);
  const uint32_t parts = c->k3_items && budget != kBudgetAll && budget >= 64u * c->k3_items ? c->k3_items : 0u;
  if (parts && !c->h_err.p) {
    HBX_TRY(c, c->h_err.ensure(64));
    std::memset(c->h_err.p, 0, 64);
  }
  if (parts)
    hipLaunchKernelGGL(hbx_k3q_block_md5, dim3(c->md5_wgs), dim3(kK3PThreads), 0, s,
                       c->d_order[slot].as<OrderEntry>(), static_cast<const uint32_t*>(c->d_octl[slot].as<uint32_t>()),
                       budget, c->d_gate.as<uint32_t>(), c->k3_dispatched, c->k3_waves + waves - 1u, tslot,
                       c->h_probe.p ? c->h_probe.as<uint64_t>() : nullptr, c->d_octl[slot].as<uint32_t>() + 1,
                       c->d_q[slot].as<uint64_t>(), (uint32_t)(L + 1), parts, c->h_err.as<uint32_t>());
  else if (c->k3_prod)
    hipLaunchKernelGGL(hbx_k3p_block_md5, dim3(c->md5_wgs), dim3(kK3PThreads), 0, s,
                       c->d_order[slot].as<OrderEntry>(), static_cast<const uint32_t*>(c->d_octl[slot].as<uint32_t>()),
                       budget, c->d_gate.as<uint32_t>(), c->k3_dispatched, c->k3_waves + waves - 1u, tslot,
                       c->h_probe.p ? c->h_probe.as<uint64_t>() : nullptr, c->k3_psets | (c->k3_spin ? 0x100u : 0u));
  else
    hipLaunchKernelGGL(hbx_k3_block_md5, dim3(c->md5_wgs), dim3(kK3Threads), 0, s,
                       c->d_order[slot].as<OrderEntry>(), static_cast<const uint32_t*>(c->d_octl[slot].as<uint32_t>()),
                       budget, c->d_gate.as<uint32_t>(), c->k3_dispatched, c->k3_waves + waves - 1u, tslot,
                       c->h_probe.p ? c->h_probe.as<uint64_t>() : nullptr);
  g_slow.mark(7);
  HBX_TRY(c, hipGetLastError());
  c->k3_dispatched += c->md5_wgs;
  c->k3_waves += waves;
  c->last_budget = budget;  // what the next plan advances this list by
  // the launch's one completion event: the plan three launches on waits for
  // it, and so does the result stream for the batches it completes
  HBX_TRY(c, hipEventRecord(c->order_free[L % kDoneRing], s));
  g_slow.mark(8);
  c->launches++;
  if (budget == kBudgetAll)  // per-batch stage times of a synchronous batch (hbx_stage_times)
    for (Batch* nb : nbs) {
      HBX_TRY(c, hipEventRecord(nb->ev[3], s));
      nb->ev3 = true;
    }
  bool forked = false;
  for (Batch* b : c->pending) {
    if (b->finalized || !b->joined) continue;
    b->done++;
    if (budget == kBudgetAll || b->done >= b->need) {
      if (!forked && c->rstream != s) {  // the result stream picks up after this K3
        HBX_TRY(c, hipStreamWaitEvent(c->rstream, c->order_free[L % kDoneRing], 0));
        forked = true;
      }
      b->final_launch = L;
      int rc = finalize_batch(c, b);
      if (rc) return rc;
    }
  }
  g_slow.mark(9);
  return HBX_OK;
}

// One pipeline step on the hash side: launch j = plan (the carried chains +
// the chains of every unjoined batch at least join_lag submits old) then K3
// with `budget` blocks per chain.  Issued by every submit BEFORE the new
// batch's own scan is enqueued (with a K3 period P, by every P-th submit
// only, with P x the slice), and by wait_oldest (`drain`, with kBudgetAll:
// the oldest unjoined batch joins whatever its age).  Nothing is launched
// when no chain is in flight.
// The unjoined batches (oldest first) that join a launch whose FIFO holds
// `size` of them, `older` submits from now: those join_lag or more old then.
uint32_t joiners(const hbx_ctx* c, uint64_t older, bool drain) {
  const uint64_t size = c->unjoined.size();
  uint64_t k = size + older >= c->join_lag ? size + older + 1 - c->join_lag : 0;
  if (drain) k = std::max<uint64_t>(k, 1);
  return (uint32_t)std::min<uint64_t>(std::min<uint64_t>(k, size), kMaxFresh);
}

int md5_step(hbx_ctx* c, uint32_t budget, bool drain = false) {
  if (!drain && c->k3_period > 1 && c->k3_tick++ % c->k3_period != 0) return HBX_OK;  // not this submit
  budget = launch_budget(c, budget);
  if (c->preplanned) {  // planned one launch ahead (mode 2): any budget may run it
    std::vector<Batch*> nbs;
    nbs.swap(c->pre_nb);
    c->preplanned = false;
    for (Batch* nb : nbs) nb->joined = true;
    return md5_launch(c, nbs, budget);
  }
  std::vector<Batch*> nbs(c->unjoined.begin(), c->unjoined.begin() + joiners(c, 0, drain));
  bool live = !nbs.empty();
  for (Batch* b : c->pending)
    if (b->joined && !b->finalized) live = true;
  if (!live) return HBX_OK;
  int rc = plan_launch(c, nbs, budget);
  if (rc) return rc;
  for (Batch* nb : nbs) {
    nb->joined = true;
    c->unjoined.pop_front();
  }
  return md5_launch(c, nbs, budget);
}

// Modes 2 and 3: enqueue the plan of the NEXT launch now, before the
// submitting batch's own K1.  It adds the unjoined batches that are join_lag
// submits old at the next submit (the submitting batch is not in the FIFO
// yet, hence `older` 1).  With a K3 period, only when the next submit
// launches.  Nothing is planned when no chain would be in flight; the next
// submit then plans inline.
int preplan(hbx_ctx* c, uint32_t budget) {
  const int mode = plan_mode_of(c);
  if ((mode != 2 && mode != 3) || c->preplanned || c->hstream == c->stream) return HBX_OK;
  if (c->k3_period > 1 && c->k3_tick % c->k3_period != 0) return HBX_OK;
  budget = launch_budget(c, budget);
  std::vector<Batch*> nbs(c->unjoined.begin(), c->unjoined.begin() + joiners(c, 1, false));
  bool live = !nbs.empty();
  for (Batch* b : c->pending)
    if (b->joined && !b->finalized) live = true;
  if (!live) return HBX_OK;
  int rc = ensure_plan_buffers(c, 0);  // its slot's last reader (K3 three launches back) is waited for
  if (!rc) rc = plan_launch(c, nbs, budget);
  if (rc) return rc;
  for (size_t i = 0; i < nbs.size(); i++) c->unjoined.pop_front();
  c->pre_nb = std::move(nbs);
  c->preplanned = true;
  return HBX_OK;
}

// The order-list and planner buffers the next launch's plan writes, with
// `extra` chains joining the unfinalized batches' chains.  Only the slot the
// plan writes may grow: growing reallocates without copying, and the slot of
// the previous launch holds the carried chains the plan reads.
int ensure_plan_buffers(hbx_ctx* c, uint64_t extra) {
  if (c->preplanned) return HBX_OK;  // that slot holds the next launch's list already
  uint64_t bound = 64 + extra;  // entries <= chains of the unfinalized batches
  for (Batch* b : c->pending)
    if (!b->finalized) bound += b->caps;
  const int slot = (int)(c->launches % 3);
  int rc = ensure_shared(c, c->d_order[slot], bound * sizeof(OrderEntry));
  if (!rc) rc = ensure_shared(c, c->d_octl[slot], 256);
  if (!rc) rc = ensure_shared(c, c->d_q[slot], (bound / 64 + 2) * 8 * 8);  // groups x up to 8 parts
  if (!rc) rc = ensure_shared(c, c->d_plan, 2 * kPlanBins * sizeof(uint32_t));
  return rc;
}

// A submit failed.  Before any device work of `b` was enqueued (`enqueued`
// false) the batch simply returns to the pool.  After it, the batch leaves
// the FIFO (so no later wait collects it into caller memory that may be
// freed), the streams drain, its buffers are parked (its chains may still be
// in the carried order lists) and the context refuses further pipelined work.
int submit_abort(hbx_ctx* c, Batch* b, int rc, bool enqueued) {
  const std::string keep = c->err;
  for (auto it = c->unjoined.begin(); it != c->unjoined.end(); ++it)
    if (*it == b) {
      c->unjoined.erase(it);
      break;
    }
  for (auto it = c->pending.begin(); it != c->pending.end(); ++it)
    if (*it == b) {
      c->pending.erase(it);
      break;
    }
  if (!enqueued) {
    c->pool.push_back(b);
    return rc;
  }
  for (hipStream_t s : {c->stream, c->cstream, c->hstream, c->rstream})
    if (s) (void)hipStreamSynchronize(s);
  c->parked.push_back(b);
  c->broken = true;
  c->err = keep + " (context is unusable for pipelined work; destroy it)";
  return rc;
}

int submit_batch_launch(hbx_ctx* c, Batch* b, const void* d_arena, uint64_t n, const uint64_t* offs,
                        const uint64_t* lens, uint32_t budget, uint64_t slices, size_t meta_bytes, int slot);

// K1 tiles of one file of `iters` 64 KiB iterations: `tile` each.
// (Queuing each file's last eighth as 1 MiB tiles after the long ones, to
// round off K1's last pass over the CUs K3 leaves free, measured slower: K1
// 3.18 -> 3.33 ms beside K3 at 33 resident batches, from the extra halos and
// workgroups.)
void k1_tiles(hbx_ctx* c, uint32_t f, uint32_t iters, uint32_t tile) {
  for (uint32_t i = 0; i < iters; i += tile) c->h_tiles.push_back(make_uint4(f, i, std::min(tile, iters - i), 0u));
}

constexpr uint32_t kTileItersMin = 16, kTileItersMax = 256;

// K1 tile length for a batch of `total` iterations (c->tile_iters, or about
// two or four tiles per CU when that is 0)
uint32_t k1_tile_iters(const hbx_ctx* c, uint64_t total) {
  if (c->tile_iters) return c->tile_iters;
  // about two tiles per CU for large batches, four up to 4 GiB (65,536
  // iterations), 8/3 up to 2 GiB: the strong-scaling shares of configs[2]
  // (tools/gpu_tile_sweep.sh, profiles/r02n_tiles: 1 GiB 1,825 -> 1,948 GiB/s
  // with 16 instead of 32 iterations, 2 GiB 2,068 -> 2,147 with 32 instead of
  // 64; 4 GiB equal; 8 GiB 2,231 at 256 vs 2,205 at 128).  With the K3 period
  // (round 5) 1 GiB does best at 24 (2,141-2,150 vs 2,096-2,132 GiB/s at 16,
  // three alternating rounds, profiles/r05s) and 2 GiB at 48 (2,275 vs 2,254)
  const uint64_t num = total <= 32768ull ? 3ull : 1ull;
  const uint64_t den = total <= 32768ull ? 8ull : total <= 65536ull ? 4ull : 2ull;
  const uint64_t t = (total * num + den * c->md5_wgs - 1) / (den * c->md5_wgs);
  return (uint32_t)std::min<uint64_t>(kTileItersMax, std::max<uint64_t>(kTileItersMin, t));
}

inline uint64_t scan_iters(uint64_t N) {  // K1 iterations of a file (0: no split candidates)
  return N > 2ull * HBX_MIN_BLOCK_SIZE ? (N + HBX_MIN_BLOCK_SIZE - 1) / HBX_MIN_BLOCK_SIZE : 0;
}

// Plan + enqueue one device batch (K1, K2, first MD5 launch).  Results are
// collected by wait_oldest in submission order.  Every validation and
// allocation happens before the batch joins the FIFO; a failure after that
// removes it again (submit_abort), so a failed submit leaves no pending batch.
int submit_batch_timed(hbx_ctx* c, const void* d_arena, uint64_t n, const uint64_t* offs,
                       const uint64_t* lens, uint64_t* cut_ends, uint8_t* ids, const uint64_t* out_base,
                       const uint64_t* caps, hbx_file_summary* sums, uint32_t budget);
}  // namespace
// hbx_reserve with the context's lock already held (defined beside it, inside
// the C-ABI block; not exported)
extern "C" __attribute__((visibility("hidden"))) int reserve_locked(hbx_ctx* c, uint32_t batches, uint64_t files,
                                                                    uint64_t bytes);
namespace {
int submit_batch(hbx_ctx* c, const void* d_arena, uint64_t n, const uint64_t* offs,
                 const uint64_t* lens, uint64_t* cut_ends, uint8_t* ids, const uint64_t* out_base,
                 const uint64_t* caps, hbx_file_summary* sums, uint32_t budget) {
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = submit_batch_timed(c, d_arena, n, offs, lens, cut_ends, ids, out_base, caps, sums, budget);
  c->max_submit_ms = std::max(c->max_submit_ms, ms_since(t0));
  return rc;
}
int submit_batch_timed(hbx_ctx* c, const void* d_arena, uint64_t n, const uint64_t* offs,
                       const uint64_t* lens, uint64_t* cut_ends, uint8_t* ids, const uint64_t* out_base,
                       const uint64_t* caps, hbx_file_summary* sums, uint32_t budget) {
  g_slow.mark(0);
  g_slow.clear();
  if (c->broken) return c->fail(HBX_ERR_STATE, "context is unusable after a failed submit; destroy it");
  if (n > 0xFFFFFFFFull) return c->fail(HBX_ERR_ARG, "too many files");
  for (uint64_t f = 0; f < n; f++)
    if (offs[f] % HBX_ARENA_ALIGN) return c->fail(HBX_ERR_ARG, "file offset not 16-byte aligned");
  Batch* b = acquire_batch(c);
  if (!b) return c->fail(HBX_ERR_HIP, "cannot create batch events");
  b->n = n;
  b->cut_ends = cut_ends;
  b->ids = ids;
  b->sums = sums;
  b->out_base.assign(out_base, out_base + n);
  b->capv.assign(caps, caps + n);
  b->cut_base.resize(n);
  c->h_slice_base.resize(n);
  c->h_tiles.clear();
  uint64_t slices = 0, tcaps = 0, longest = 0, total_iters = 0;
  for (uint64_t f = 0; f < n; f++) {
    const uint64_t iters = scan_iters(lens[f]);
    if (iters > 0xFFFFFFFFull) {
      c->pool.push_back(b);
      return c->fail(HBX_ERR_ARG, "file too large");
    }
    total_iters += iters;
  }
  const uint32_t tile = k1_tile_iters(c, total_iters);
  for (uint64_t f = 0; f < n; f++) {
    const uint64_t N = lens[f];
    longest = std::max(longest, N);
    c->h_slice_base[f] = slices;
    b->cut_base[f] = tcaps;
    tcaps += max_chunks(N);
    if (const uint64_t iters = scan_iters(N)) {  // only files with split candidates scan
      slices += (N + kSlice - 1) / kSlice;
      k1_tiles(c, (uint32_t)f, (uint32_t)iters, tile);
    }
  }
  b->caps = tcaps;
  // launches this batch's chains need: a chunk is <= min(longest file, MAX)
  // bytes, i.e. <= nfull full message blocks, and each launch advances it by
  // slice_cnt(remaining, budget) blocks (the part short of a slice first, then
  // full slices): ceil(blocks / budget) launches either way
  const uint64_t nfull = (std::min<uint64_t>(longest, HBX_MAX_BLOCK_SIZE) + 8) >> 6;
  const uint64_t lb = launch_budget(c, budget);  // a K3 period multiplies the slice
  b->need = budget == kBudgetAll ? 1u : (uint32_t)std::max<uint64_t>(1, (nfull + lb - 1) / lb);
  const uint64_t nt = c->h_tiles.size();
  // meta block: off | len | slice_base | cut_base | tiles
  const size_t meta_bytes = n * 8 * 4 + nt * sizeof(uint4);
  const int slot = c->ssum_slot;
  g_slow.mark(1);
  if (n) {  // every allocation first: the batch is not in the FIFO yet
    int rc = HBX_OK;
    b->rl = res_layout(n, tcaps);
    for (hipError_t e : {b->h_meta.ensure(meta_bytes), b->d_meta.ensure(meta_bytes), b->d_res.ensure(b->rl.total),
                         b->d_run.ensure(tcaps * sizeof(Chain)),
                         b->d_fresh.ensure(tcaps * sizeof(OrderEntry)), b->d_fcnt.ensure(256),
                         b->h_res.ensure(b->rl.total)})
      if (e != hipSuccess && !rc) rc = c->hip(e, "batch buffers");
    if (!rc) rc = ensure_shared(c, c->d_ssum[slot], (slices + 1) * sizeof(uint2));  // +1: dummy slot
    if (!rc) rc = ensure_plan_buffers(c, tcaps);
    if (rc) return submit_abort(c, b, rc, false);
  }
  c->pending.push_back(b);
  g_slow.mark(2);
  const int rc = submit_batch_launch(c, b, d_arena, n, offs, lens, budget, slices, meta_bytes, slot);
  g_slow.mark(5);
  g_slow.report(c->launches);
  return rc ? submit_abort(c, b, rc, true) : HBX_OK;
}

int submit_batch_launch(hbx_ctx* c, Batch* b, const void* d_arena, uint64_t n, const uint64_t* offs,
                        const uint64_t* lens, uint32_t budget, uint64_t slices, size_t meta_bytes, int slot) {
  hipStream_t s = c->stream;
  // launch j hashes the chains in flight plus the previous batch's; it is
  // enqueued (plan on the scan stream) before this batch's K1, so it never
  // waits for this batch's scan
  const uint64_t launches0 = c->launches;
  int rc = md5_step(c, budget);
  g_slow.mark(3);
  if (!rc) rc = preplan(c, budget);
  g_slow.mark(4);
  if (rc) return rc;
  const bool gate = c->k1_gate && c->launches != launches0 && c->hstream != s;
  if (n == 0) {
    for (int i = 0; i < 4; i++) HBX_TRY(c, hipEventRecord(b->ev[i], s));
    b->finalized = true;
    HBX_TRY(c, hipEventRecord(b->ev[4], s));
    return HBX_OK;
  }
  const uint64_t nt = c->h_tiles.size();
  uint64_t* hm = b->h_meta.as<uint64_t>();
  std::memcpy(hm, offs, n * 8);
  std::memcpy(hm + n, lens, n * 8);
  std::memcpy(hm + 2 * n, c->h_slice_base.data(), n * 8);
  std::memcpy(hm + 3 * n, b->cut_base.data(), n * 8);
  if (nt) std::memcpy(hm + 4 * n, c->h_tiles.data(), nt * sizeof(uint4));
  c->ssum_slot ^= 1;
  DevBuf& ssum = c->d_ssum[slot];

  if (int frc = flush_input_wait(c)) return frc;  // (no launch this submit: nothing flushed it yet)
  const bool gate_meta = c->meta_kernel && c->gate_meta && c->k1_gate;
  if (gate_meta) {  // one kernel: the meta copy, then (if a K3 launch was issued) the gate
    if (c->ssum_used[slot] && c->cstream != s) HBX_TRY(c, hipStreamWaitEvent(s, c->ssum_free[slot], 0));
    const uint32_t n16 = (uint32_t)(meta_bytes / 16);
    hipLaunchKernelGGL(hbx_k1_gate_meta, dim3(std::min<uint32_t>(16, (n16 + 255) / 256)), dim3(256), 0, s,
                       static_cast<const uint32_t*>(c->d_gate.as<uint32_t>()), c->k3_dispatched, 1000000u,
                       gate ? 1u : 0u, static_cast<const uint4*>(b->h_meta.p), b->d_meta.as<uint4>(), n16);
    HBX_TRY(c, hipGetLastError());
  } else if (c->meta_kernel) {  // meta_bytes is a multiple of 16
    const uint32_t n16 = (uint32_t)(meta_bytes / 16);
    hipLaunchKernelGGL(hbx_meta_fetch, dim3(std::min<uint32_t>(64, (n16 + 255) / 256)), dim3(256), 0, s,
                       static_cast<const uint4*>(b->h_meta.p), b->d_meta.as<uint4>(), n16);
    HBX_TRY(c, hipGetLastError());
  } else {
    HBX_TRY(c, hipMemcpyAsync(b->d_meta.p, hm, meta_bytes, hipMemcpyHostToDevice, s));
  }
  const uint64_t* d_off = b->d_meta.as<uint64_t>();
  const uint64_t* d_len = d_off + n;
  const uint64_t* d_sb = d_off + 2 * n;
  const uint64_t* d_cb = d_off + 3 * n;
  const uint4* d_tiles = reinterpret_cast<const uint4*>(d_off + 4 * n);
  const uint8_t* arena = static_cast<const uint8_t*>(d_arena);

  // the K2 that last read this summary slot (two batches back) must be done
  if (!gate_meta && c->ssum_used[slot] && c->cstream != s) HBX_TRY(c, hipStreamWaitEvent(s, c->ssum_free[slot], 0));
  if (gate && !gate_meta) {  // K1 after the K3 launch above has all its workgroups on CUs (<= 10 ms)
    hipLaunchKernelGGL(hbx_k1_gate, dim3(1), dim3(64), 0, s, static_cast<const uint32_t*>(c->d_gate.as<uint32_t>()),
                       c->k3_dispatched, 1000000u);
    HBX_TRY(c, hipGetLastError());
  }
  // lean marks with K2 on this stream: ev[0] | K1 | ev[1] | K2 | ev[5] | K2r
  // (| ev[2] unless the plan follows on this stream), one record between
  // kernels, the batch's events doubling as K1's
  // and K2's timers (the batch outlives their harvest: it is reused only
  // after its collect, long after both completed)
  hipStream_t s2 = c->cstream;
  const bool lean = c->lean_marks && s2 == s;
  if (nt && c->k1_ext) {
    // round 6: ev[0] / ev[1] bound to K1's own dispatch (hipExtLaunchKernel's
    // start and stop events), not recorded as marker packets around it: at
    // join lag >= 2 K1 had four (ev[0], its timer's pair, ev[1]) between the
    // scan loop's kernels.  They double as K1's timer and K2's dependency.
    hipExtLaunchKernelGGL(hbx_k1_digest_scan_dma, dim3((uint32_t)nt), dim3(kK1Threads), 0, s, b->ev[0], b->ev[1], 0,
                          arena, d_off, d_len, d_sb, d_tiles, ssum.as<uint2>(), slices,
                          c->k1_swz | (c->k1_dma4 ? 0u : 2u) | (c->k1_early ? 0u : 4u));
    HBX_TRY(c, hipGetLastError());
    c->open_t.push_back(TimedLaunch{b->ev[0], b->ev[1], 0, false});
  } else {
    HBX_TRY(c, hipEventRecord(b->ev[0], s));
    if (nt) {
      StageTimer t(c, s, 0, !lean);
      hipLaunchKernelGGL(hbx_k1_digest_scan_dma, dim3((uint32_t)nt), dim3(kK1Threads), 0, s, arena, d_off, d_len,
                         d_sb, d_tiles, ssum.as<uint2>(), slices, c->k1_swz | (c->k1_dma4 ? 0u : 2u) | (c->k1_early ? 0u : 4u));
    }
    HBX_TRY(c, hipGetLastError());
    HBX_TRY(c, hipEventRecord(b->ev[1], s));
    if (lean && nt) c->open_t.push_back(TimedLaunch{b->ev[0], b->ev[1], 0, false});
  }
  // K2 on the cut stream: the scan stream goes straight on with the next
  // batch's K1 (into the other summary slot)
  if (s2 != s) HBX_TRY(c, hipStreamWaitEvent(s2, b->ev[1], 0));
  {
    StageTimer t(c, s2, 1, !lean);
    hipLaunchKernelGGL(hbx_k2_cut_chain, dim3((uint32_t)n), dim3(64), 0, s2, arena, d_off, d_len,
                       d_sb, ssum.as<uint2>(), d_cb, b->cuts_d(), b->count_d(),
                       lean ? b->d_fcnt.as<uint32_t>() : nullptr);
  }
  HBX_TRY(c, hipGetLastError());
  if (lean) {  // the summary slot's next writer (K1, this stream) follows in order: no ssum_free
    HBX_TRY(c, hipEventRecord(b->ev[5], s2));
    c->open_t.push_back(TimedLaunch{b->ev[1], b->ev[5], 1, false});
  } else {
    HBX_TRY(c, hipEventRecord(c->ssum_free[slot], s2));
  }
  c->ssum_used[slot] = true;
  // K2r: the batch's chains and their order entries (lean: K2 zeroed the count)
  if (!lean) HBX_TRY(c, hipMemsetAsync(b->d_fcnt.p, 0, 4, s2));
  hipLaunchKernelGGL(hbx_k2r_new_chains, dim3((uint32_t)((n * kPlanLanesPerFile + 255) / 256)), dim3(256), 0, s2,
                     (uint32_t)n, arena, d_off, d_cb, b->cuts_d(), b->count_d(), b->ids_d(), b->d_run.as<Chain>(), b->d_fresh.as<OrderEntry>(),
                     b->d_fcnt.as<uint32_t>());
  HBX_TRY(c, hipGetLastError());
  // the plan this batch joins waits for ev[2] (plan_launch), so with a join
  // lag of 2 the scan stream never waits for this K2.  Lean marks with the
  // plan on this same stream: no one waits, and ev[5] already marks K2's end
  if (lean && plan_stream(c) == s2) {
    b->k2_ev5 = true;
  } else {
    HBX_TRY(c, hipEventRecord(b->ev[2], s2));
  }
  c->unjoined.push_back(b);
  return HBX_OK;
}

int submit_verify_launch(hbx_ctx* c, Batch* b, const uint8_t* arena, uint64_t n, const uint64_t* offs,
                         const uint64_t* lens, const uint8_t* links, const uint64_t* link_base,
                         const uint32_t* n_links, uint64_t nlinks_total, size_t meta_bytes, uint32_t budget);

// Plan + enqueue a VerifyBlock batch: K6p hashes each block's prefix blocks
// and turns the rest into K3 chains, which then share the time-sliced MD5
// pipeline (and the FIFO of hbx_wait) with the chunking batches.
int submit_verify(hbx_ctx* c, const uint8_t* arena, uint64_t n, const uint64_t* offs, const uint64_t* lens,
                  const uint8_t* links, const uint64_t* link_base, const uint32_t* n_links, uint8_t* ids,
                  const uint8_t* expect, uint8_t* ok, uint64_t* n_bad, uint32_t budget) {
  if (c->broken) return c->fail(HBX_ERR_STATE, "context is unusable after a failed submit; destroy it");
  if (n > 0xFFFFFFFFull) return c->fail(HBX_ERR_ARG, "too many blocks");
  uint64_t nlinks_total = 0, longest = 0;
  for (uint64_t i = 0; i < n; i++) {
    const uint32_t nl = n_links ? n_links[i] : 0u;
    if (nl && (!links || !link_base)) return c->fail(HBX_ERR_ARG, "links missing");
    if (lens[i] + 8ull + 16ull * nl + 128ull > 0xFFFFFFFFull) return c->fail(HBX_ERR_ARG, "block too large");
    if (nl) nlinks_total = std::max(nlinks_total, link_base[i] + nl);
    longest = std::max<uint64_t>(longest, (lens[i] + 8ull + 16ull * nl) >> 6);
  }
  Batch* b = acquire_batch(c);
  if (!b) return c->fail(HBX_ERR_HIP, "cannot create batch events");
  b->verify = true;
  b->n = n;
  b->caps = n;
  b->v_ids = ids;
  b->v_expect = expect;
  b->v_ok = ok;
  b->v_nbad = n_bad;
  const uint64_t lb = launch_budget(c, budget);
  b->need = budget == kBudgetAll ? 1u : (uint32_t)std::max<uint64_t>(1, (longest + lb - 1) / lb);
  // meta block: descriptors | links
  const size_t meta_bytes = n * sizeof(VerifyDesc) + 16 * nlinks_total;
  if (n) {  // every allocation first: the batch is not in the FIFO yet
    int rc = HBX_OK;
    for (hipError_t e : {b->h_meta.ensure(meta_bytes), b->d_meta.ensure(meta_bytes), b->d_res.ensure(n * 16),
                         b->d_run.ensure(n * sizeof(Chain)), b->d_fresh.ensure(n * sizeof(OrderEntry)),
                         b->d_fcnt.ensure(256), b->h_res.ensure(n * 16)})
      if (e != hipSuccess && !rc) rc = c->hip(e, "verify batch buffers");
    if (!rc) rc = ensure_plan_buffers(c, n);
    if (rc) return submit_abort(c, b, rc, false);
  }
  c->pending.push_back(b);
  const int rc = submit_verify_launch(c, b, arena, n, offs, lens, links, link_base, n_links, nlinks_total,
                                      meta_bytes, budget);
  return rc ? submit_abort(c, b, rc, true) : HBX_OK;
}

int submit_verify_launch(hbx_ctx* c, Batch* b, const uint8_t* arena, uint64_t n, const uint64_t* offs,
                         const uint64_t* lens, const uint8_t* links, const uint64_t* link_base,
                         const uint32_t* n_links, uint64_t nlinks_total, size_t meta_bytes, uint32_t budget) {
  hipStream_t s = c->stream;
  int rc = md5_step(c, budget);  // launch j first, as in submit_batch_launch
  if (!rc) rc = preplan(c, budget);
  if (!rc) rc = flush_input_wait(c);
  if (rc) return rc;
  if (n == 0) {
    for (int i = 0; i < 4; i++) HBX_TRY(c, hipEventRecord(b->ev[i], s));
    b->finalized = true;
    HBX_TRY(c, hipEventRecord(b->ev[4], s));
    return HBX_OK;
  }
  VerifyDesc* hd = b->h_meta.as<VerifyDesc>();
  uint8_t* dl = b->d_meta.as<uint8_t>() + n * sizeof(VerifyDesc);
  for (uint64_t i = 0; i < n; i++) {
    const uint32_t nl = n_links ? n_links[i] : 0u;
    hd[i].src = reinterpret_cast<uint64_t>(arena + offs[i]);
    hd[i].links = reinterpret_cast<uint64_t>(dl + (nl ? 16 * link_base[i] : 0));
    hd[i].len = (uint32_t)lens[i];
    hd[i].n_links = nl;
    hd[i].pad = 0;
  }
  if (nlinks_total) std::memcpy(b->h_meta.as<uint8_t>() + n * sizeof(VerifyDesc), links, 16 * nlinks_total);
  HBX_TRY(c, hipEventRecord(b->ev[0], s));
  HBX_TRY(c, hipMemcpyAsync(b->d_meta.p, b->h_meta.p, meta_bytes, hipMemcpyHostToDevice, s));
  HBX_TRY(c, hipMemsetAsync(b->d_fcnt.p, 0, 4, s));
  HBX_TRY(c, hipEventRecord(b->ev[1], s));
  hipLaunchKernelGGL(hbx_k6p_verify_chains, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s,
                     b->d_meta.as<VerifyDesc>(), (uint32_t)n, b->ids_d(), b->d_run.as<Chain>(),
                     b->d_fresh.as<OrderEntry>(), b->d_fcnt.as<uint32_t>());
  HBX_TRY(c, hipGetLastError());
  HBX_TRY(c, hipEventRecord(b->ev[2], s));
  c->unjoined.push_back(b);
  return HBX_OK;
}

// Scatter a collected batch's pinned results into the caller's arrays.
int collect_batch(hbx_ctx* c, Batch* b) {
  const uint64_t n = b->n;
  if (b->verify) {  // VerifyBlock: ids, and the comparison with the expected ids
    const uint8_t* hid = b->h_res.as<uint8_t>();
    if (b->v_ids && n) std::memcpy(b->v_ids, hid, n * 16);
    uint64_t bad = 0;
    if (b->v_expect) {
      for (uint64_t i = 0; i < n; i++) {
        const uint8_t good = std::memcmp(hid + 16 * i, b->v_expect + 16 * i, 16) == 0;
        if (b->v_ok) b->v_ok[i] = good;
        bad += good ? 0 : 1;
      }
    }
    if (b->v_nbad) *b->v_nbad = bad;
    return HBX_OK;
  }
  const ResLayout& rl = b->rl;
  const uint8_t* hr = b->h_res.as<uint8_t>();
  const uint32_t* counts = reinterpret_cast<const uint32_t*>(hr + rl.counts);
  const uint64_t* cuts = reinterpret_cast<const uint64_t*>(hr + rl.cuts);
  const uint8_t* hid = hr + rl.ids;
  const uint8_t* cid = hr + rl.cid;
  const int32_t* ctype = reinterpret_cast<const int32_t*>(hr + rl.ctype);
  int rc = HBX_OK;
  for (uint64_t f = 0; f < n; f++) {
    const uint64_t k = counts[f];
    const uint64_t ib = b->cut_base[f];
    if (b->sums) {
      std::memcpy(b->sums[f].content_id, cid + 16 * f, 16);
      b->sums[f].content_type = ctype[f];
      b->sums[f].n_chunks = (uint32_t)k;
    }
    if (k > b->capv[f]) {
      rc = c->fail(HBX_ERR_CAPACITY, "output capacity too small for file " + std::to_string(f));
      continue;
    }
    if (b->cut_ends) std::memcpy(b->cut_ends + b->out_base[f], cuts + ib, k * 8);
    if (b->ids) std::memcpy(b->ids + 16 * b->out_base[f], hid + 16 * ib, k * 16);
  }
  float ms = 0.f;
  // stage boundaries: K1 start | K1 end | K2 end | plan+K3 end | results
  // ready (K2's end is ev[5] where lean marks left ev[2] unrecorded)
  const hipEvent_t bd[5] = {b->ev[0], b->ev[1], b->k2_ev5 ? b->ev[5] : b->ev[2], b->ev[3], b->ev[4]};
  for (int i = 0; i < 4; i++) {
    c->stage_ms[i] = 0.f;
    // a pipelined batch has no ev[3]: [2] then spans K2 end -> results ready
    const int e = (i == 2 && !b->ev3) ? 4 : i + 1;
    if ((i != 3 || b->ev3) && hipEventElapsedTime(&ms, bd[i], bd[e]) == hipSuccess) c->stage_ms[i] = ms;
  }
  if (hipEventElapsedTime(&ms, b->ev[0], b->ev[4]) == hipSuccess) c->stage_ms[4] = ms;
  return rc;
}

// Complete the oldest pending batch (draining the MD5 chains first if its
// chains are not yet guaranteed hashed) and collect it.
int wait_oldest(hbx_ctx* c) {
  if (c->pending.empty()) return HBX_OK;
  Batch* b = c->pending.front();
  if (c->broken) {  // drop it uncollected: its results are never written to the caller
    c->pending.pop_front();
    c->parked.push_back(b);
    return c->fail(HBX_ERR_STATE, "context is unusable after a failed submit; destroy it");
  }
  // drain: every chain in flight; a pre-planned launch runs first (with an
  // unlimited budget), then b joins if it had not yet (b is the oldest)
  for (int k = 0; !b->finalized; k++) {
    const uint64_t l0 = c->launches;
    int rc = md5_step(c, kBudgetAll, true);
    if (rc) return rc;
    if (c->launches == l0 || k > 2) return c->fail(HBX_ERR_STATE, "drain launched nothing (internal)");
  }
  HBX_TRY(c, hipEventSynchronize(b->ev[4]));
  if (c->h_err.p && *static_cast<volatile uint32_t*>(c->h_err.p)) {  // a K3Q wave gave up: results wrong
    c->pending.pop_front();
    c->parked.push_back(b);
    c->broken = true;
    return c->fail(HBX_ERR_STATE, "K3 item queue: a wave timed out waiting for an item (internal); destroy the context");
  }
  c->pending.pop_front();
  // ev[4] follows the K3 launch that finalized b (the result stream waited for it)
  if (b->joined) c->k3_done_upto = std::max<uint64_t>(c->k3_done_upto, b->final_launch + 1);
  int rc = collect_batch(c, b);
  c->pool.push_back(b);
  harvest_timings(c);
  harvest_k3(c);
  return rc;
}

int run_device_sync(hbx_ctx* c, const void* d_arena, uint64_t n, const uint64_t* offs,
                    const uint64_t* lens, uint64_t* cut_ends, uint8_t* ids,
                    const uint64_t* out_base, const uint64_t* caps, hbx_file_summary* sums) {
  int rc = submit_batch(c, d_arena, n, offs, lens, cut_ends, ids, out_base, caps, sums, kBudgetAll);
  if (rc) return rc;
  return wait_oldest(c);
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

// A/B and diagnostic switches (HBX_*) are read only when HBX_AB=1 is set as
// well: a caller's stray environment must not change the product path.  The
// effective values are reported by hbx_knobs().
static const char* ab_env(const char* name) {
  const char* ab = std::getenv("HBX_AB");
  return (ab && std::atoi(ab) != 0) ? std::getenv(name) : nullptr;
}

// HBX_SCAN_CUS / HBX_HASH_CUS / HBX_RES_CUS = "first:count[:stride]" restrict a
// stream's dispatches to those CU indices (hipExtStreamCreateWithCUMask);
// "off" or unset = an ordinary stream.  The scan stream defaults to a full
// mask: a CU-masked stream gets a hardware queue of its own, and K1/K2 on it
// beside K3 run 2.6 % faster end to end (2,100 vs 2,046 GiB/s, 3 A/B pairs,
// tools/gpu_ab_cumask3.sh).  Masking the hash or result stream, even with
// all CUs, serializes K1 and K3 (1,510-1,540 GiB/s): leave them unmasked.
static hipError_t make_stream(hipStream_t* s, const char* env, int ncu, const char* dflt = nullptr) {
  const char* v = ab_env(env);
  if (!v) v = dflt;
  int first = 0, count = 0, stride = 1;
  if (!v || std::sscanf(v, "%d:%d:%d", &first, &count, &stride) < 2 || count <= 0 || ncu <= 0) {
    // A/B only: "prio:hi" / "prio:lo" = an unmasked stream at the device's
    // greatest / least priority
    int lo = 0, hi = 0;
    if (v && std::strncmp(v, "prio:", 5) == 0 && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess)
      return hipStreamCreateWithPriority(s, hipStreamNonBlocking, std::strcmp(v + 5, "hi") == 0 ? hi : lo);
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  }
  std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
  for (int i = 0, cu = first; i < count && cu < ncu; i++, cu += std::max(1, stride))
    mask[(size_t)cu / 32] |= 1u << (cu % 32);
  // the mask is a scheduling choice, not a requirement: a runtime that
  // refuses it gets an ordinary stream
  if (hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data()) == hipSuccess) return hipSuccess;
  (void)hipGetLastError();
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

// SDMA engine warm-up (verdict r05 item 2: the ~7 ms host stall in the copy
// call).  The HSA runtime creates an SDMA engine's queue the first time a
// copy is put on that engine, and hipMemcpyAsync puts a copy on the first
// engine that is free at the call: with one 8 GiB H2D copy still running the
// next goes to the next engine, so the first copies of a pipeline each met a
// fresh engine and the call held the host 7.2-7.6 ms while the runtime
// built its queue (AMD_LOG_LEVEL=4 of the e2e leg: only the first 8 GiB copy on
// engines 0x2, 0x4, 0x8 and 0x10 was slow, every later one on the same engine
// took 17-34 us; HSA_ENABLE_SDMA=0 removed the stall with blit kernels,
// ROC_SIGNAL_POOL_SIZE and HSA_ENABLE_SDMA_GANG did not move it;
// profiles/r06c).  So every engine the runtime reports for H2D and D2H gets
// one 64-byte copy here, once per device per process, before any pipeline
// runs.  HBX_SDMA_WARM=0 (A/B) leaves the engines cold.
static hsa_status_t first_cpu_agent(hsa_agent_t a, void* data) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t*>(data) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}
static void warm_sdma_engines(hbx_ctx* c) {
  static std::mutex mu;
  static uint64_t done = 0;  // devices warmed in this process (bit per device)
  std::lock_guard<std::mutex> g(mu);
  if (c->device >= 64 || (done >> c->device) & 1u) return;
  const auto t0 = std::chrono::steady_clock::now();
  void* d = nullptr;
  void* h = nullptr;
  if (hipMalloc(&d, 4096) != hipSuccess || hipHostMalloc(&h, 4096, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    if (d) (void)hipFree(d);
    return;  // no warm-up: correct, only the first copies per engine are slow
  }
  std::memset(h, 0, 4096);
  hsa_amd_pointer_info_t pi;
  std::memset(&pi, 0, sizeof(pi));
  pi.size = sizeof(pi);
  hsa_agent_t cpu{0};
  hsa_signal_t sig{0};
  if (hsa_amd_pointer_info(d, &pi, nullptr, nullptr, nullptr) == HSA_STATUS_SUCCESS && pi.agentOwner.handle &&
      hsa_iterate_agents(first_cpu_agent, &cpu) != HSA_STATUS_ERROR && cpu.handle &&
      hsa_signal_create(1, 0, nullptr, &sig) == HSA_STATUS_SUCCESS) {
    const hsa_agent_t gpu = pi.agentOwner;
    for (int dir = 0; dir < 2; dir++) {
      const hsa_agent_t dst = dir ? cpu : gpu, src = dir ? gpu : cpu;
      uint32_t mask = 0;
      if (hsa_amd_memory_copy_engine_status(dst, src, &mask) != HSA_STATUS_SUCCESS) continue;
      (dir ? c->sdma_d2h : c->sdma_h2d) = mask;
      for (uint32_t bit = 1; bit && bit <= mask; bit <<= 1) {
        if (!(mask & bit)) continue;
        hsa_signal_store_screlease(sig, 1);
        if (hsa_amd_memory_async_copy_on_engine(dir ? h : d, dst, dir ? d : h, src, 64, 0, nullptr, sig,
                                                (hsa_amd_sdma_engine_id_t)bit, true) != HSA_STATUS_SUCCESS)
          continue;
        (void)hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
      }
    }
    hsa_signal_destroy(sig);
  }
  (void)hipHostFree(h);
  (void)hipFree(d);
  done |= 1ull << c->device;
  c->sdma_warm_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int hbx_ctx_create(int device, hbx_ctx** out) {
  if (!out) return HBX_ERR_ARG;
  *out = nullptr;
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0) return HBX_ERR_NODEV;
  if (device < 0 || device >= nd) return HBX_ERR_ARG;
  hbx_ctx* c = new hbx_ctx();
  c->device = device;
  hipDeviceProp_t prop;
  int ncu = 0;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    c->md5_wgs = (uint32_t)(ncu = prop.multiProcessorCount);
  if (const char* v = ab_env("HBX_TILE_ITERS")) c->tile_iters = (uint32_t)std::min(1024, std::max(0, std::atoi(v)));
  if (const char* v = ab_env("HBX_K3_PERIOD")) c->k3_period = (uint32_t)std::min(kMaxFresh, std::max(1, std::atoi(v)));
  if (const char* v = ab_env("HBX_JOIN_LAG")) c->join_lag = (uint32_t)std::min(4, std::max(1, std::atoi(v)));
  if (const char* v = ab_env("HBX_K4_WINDOW")) c->k4_window = (uint32_t)std::min(1024, std::max(1, std::atoi(v)));
  if (const char* v = ab_env("HBX_MD5_SLICE")) c->md5_slice = (uint32_t)std::max(0, std::atoi(v));
  if (const char* v = ab_env("HBX_K1_GATE")) c->k1_gate = std::atoi(v) ? 1u : 0u;
  if (const char* v = ab_env("HBX_LEAN_MARKS")) c->lean_marks = std::atoi(v) ? 1u : 0u;
  if (const char* v = ab_env("HBX_D2H_KERNEL")) c->d2h_kernel = (uint32_t)std::min(std::max(std::atoi(v), 0), 1024);
  if (const char* v = ab_env("HBX_K3_PROD")) c->k3_prod = std::atoi(v) ? 1u : 0u;
  if (const char* v = ab_env("HBX_PLAN_CUT")) c->plan_cut = (uint32_t)std::min(2, std::max(0, std::atoi(v)));
  if (const char* v = ab_env("HBX_META_KERNEL")) c->meta_kernel = std::atoi(v) ? 1u : 0u;
  if (const char* v = ab_env("HBX_GATE_META")) c->gate_meta = std::atoi(v) ? 1u : 0u;
  if (const char* v = ab_env("HBX_SDMA_WARM")) c->sdma_warm = std::atoi(v) ? 1u : 0u;
  if (const char* v = ab_env("HBX_K3_PSETS")) c->k3_psets = std::atoi(v) == 3 ? 3u : 2u;
  if (const char* v = ab_env("HBX_K3_SPIN")) c->k3_spin = std::atoi(v) ? 1u : 0u;
  if (const char* v = ab_env("HBX_PLAN_ADDR")) c->plan_addr = (uint32_t)std::min(512, std::max(0, std::atoi(v)));
  if (const char* v = ab_env("HBX_PLAN_ADDR_SHIFT")) c->plan_addr_shift = (uint32_t)std::min(40, std::max(20, std::atoi(v)));
  if (const char* v = ab_env("HBX_K1_EXT")) c->k1_ext = std::atoi(v) ? 1u : 0u;
  if (const char* v = ab_env("HBX_K1_DMA4")) c->k1_dma4 = std::atoi(v) ? 1u : 0u;
  if (const char* v = ab_env("HBX_K1_EARLY")) c->k1_early = std::atoi(v) ? 1u : 0u;
  if (const char* v = ab_env("HBX_K1_SWZ")) c->k1_swz = std::atoi(v) ? 1u : 0u;
  if (const char* v = ab_env("HBX_K3_ITEMS")) c->k3_items = (uint32_t)std::min(8, std::max(0, std::atoi(v)));
  // (tests: a K3 grid of a few workgroups, so every wave takes many groups)
  if (const char* v = ab_env("HBX_K3_WGS")) c->md5_wgs = (uint32_t)std::min<int>(std::max(1, ncu), std::max(1, std::atoi(v)));
  if (hipSetDevice(device) != hipSuccess || make_stream(&c->stream, "HBX_SCAN_CUS", ncu, "0:4096") != hipSuccess) {
    delete c;
    return HBX_ERR_HIP;
  }
  if (const char* v = ab_env("HBX_K2_STREAM")) c->k2_own = std::atoi(v) ? 1 : 0;
  c->cstream = c->stream;
  if (make_stream(&c->hstream, "HBX_HASH_CUS", ncu) != hipSuccess ||
             make_stream(&c->rstream, "HBX_RES_CUS", ncu) != hipSuccess || ensure_cut_stream(c) != HBX_OK) {
    hbx_ctx_destroy(c);
    return HBX_ERR_HIP;
  }
  if (c->h_k3t.ensure(kK3TimeRing * 16) == hipSuccess) std::memset(c->h_k3t.p, 0, kK3TimeRing * 16);
  if (c->d_gate.ensure(256) != hipSuccess || hipMemset(c->d_gate.p, 0, 256) != hipSuccess ||
      hipEventCreateWithFlags(&c->ssum_free[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ssum_free[1], hipEventDisableTiming) != hipSuccess) {
    hbx_ctx_destroy(c);
    return HBX_ERR_HIP;
  }
  for (int t = 0; t < kDoneRing; t++) {
    if ((t >= 3 || hipEventCreateWithFlags(&c->plan_done[t], hipEventDisableTiming) == hipSuccess) &&
        hipEventCreateWithFlags(&c->order_free[t], hipEventDisableTiming) == hipSuccess)
      continue;
    hbx_ctx_destroy(c);
    return HBX_ERR_HIP;
  }
  if (c->sdma_warm) warm_sdma_engines(c);
  *out = c;
  return HBX_OK;
}

void hbx_ctx_destroy(hbx_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  for (hipStream_t s : {c->stream, c->cstream, c->hstream, c->rstream})
    if (s) (void)hipStreamSynchronize(s);
  for (hipEvent_t e : {c->producer, c->ssum_free[0], c->ssum_free[1], c->plan_done[0], c->plan_done[1],
                       c->plan_done[2]})
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->order_free)
    if (e) (void)hipEventDestroy(e);
  for (DevBuf* b : {&c->d_ssum[0], &c->d_ssum[1], &c->d_order[0], &c->d_order[1], &c->d_order[2],
                    &c->d_octl[0], &c->d_octl[1], &c->d_octl[2], &c->d_q[0], &c->d_q[1], &c->d_q[2], &c->d_gate,
                    &c->d_stage, &c->d_msg, &c->d_plan, &c->d_vdesc, &c->d_vlinks,
                    &c->d_vout, &c->d_vexp, &c->d_zeros, &c->d_zblk, &c->d_zinfo, &c->d_zoff,
                    &c->d_zlen, &c->d_zout, &c->d_zimg, &c->d_idesc, &c->d_ires, &c->d_sreg, &c->d_sstart,
                    &c->d_sres, &c->d_sscratch, &c->d_smeta})
    b->release();
  for (PinBuf& h : c->h_read) h.release();
  c->h_zstage.release();
  for (auto& z : c->zs)
    if (z.stream) (void)hipStreamSynchronize(z.stream);
  for (auto& z : c->zs) {
    for (DevBuf* b : {&z.blk, &z.info, &z.off, &z.len, &z.img, &z.out}) b->release();
    z.desc.release();
    z.lens.release();
    z.stage.release();
    if (z.done) (void)hipEventDestroy(z.done);
    if (z.stream) (void)hipStreamDestroy(z.stream);
  }
  c->h_k3t.release();
  c->h_probe.release();
  c->h_err.release();
  for (DevBuf& d : c->d_ring) d.release();
  for (hipEvent_t e : c->h2d_done)
    if (e) (void)hipEventDestroy(e);
  for (Batch* b : c->pending) c->pool.push_back(b);
  for (Batch* b : c->parked) c->pool.push_back(b);
  for (Batch* b : c->pool) {
    b->release();
    delete b;
  }
  for (int i = 0; i < 3; i++)
    if (c->plan_timer_set[i]) c->open_t.push_back(c->plan_timer[i]);
  for (TimedLaunch& t : c->open_t) {
    if (!t.owned) continue;  // a batch's own events (released with the batch)
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
  for (hipStream_t s : {c->cstream, c->hstream, c->rstream})
    if (s && s != c->stream) (void)hipStreamDestroy(s);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

// Failures of calls made without a context (hbx_plan_pipeline with ctx NULL)
// are described per thread.
static thread_local std::string g_noctx_err;
const char* hbx_last_error(const hbx_ctx* c) {
  return c ? c->err.c_str() : g_noctx_err.empty() ? "null context" : g_noctx_err.c_str();
}

int hbx_set_tile_iters(hbx_ctx* c, uint32_t iters) {
  if (!c || iters > 1024) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  c->tile_iters = iters;
  return HBX_OK;
}

int hbx_set_join_lag(hbx_ctx* c, uint32_t lag) {
  if (!c || lag < 1 || lag > 4) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  // pending batches were counted against the lag of their submit
  if (!c->pending.empty()) return c->fail(HBX_ERR_STATE, "submitted batches are still pending");
  HBX_TRY(c, hipSetDevice(c->device));
  c->join_lag = lag;
  return ensure_cut_stream(c);
}

int hbx_set_k3_period(hbx_ctx* c, uint32_t period) {
  if (!c || period < 1 || period > (uint32_t)kMaxFresh) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  // pending batches were counted against the launch budget of their submit
  if (!c->pending.empty()) return c->fail(HBX_ERR_STATE, "submitted batches are still pending");
  c->k3_period = period;
  c->k3_tick = 0;
  return HBX_OK;
}

// The pipeline's operating point (DESIGN.md §3 "Throughput model", §7):
// throughput ~ bytes resident / a batch's lifetime, so R = as many arenas as
// hbm_frac of the free memory holds; a batch holds its arena for its `need`
// launches (period P apart) plus the join lag and lead, so the slice is the
// longest chain's blocks over the launches that fit in R - lead - (P - 1)
// submits.  bench.py takes every plan from here (tests/test_plan.py checks
// it against the round-5 Python planner at N = 1..8).
int hbx_plan_pipeline(hbx_ctx* c, const hbx_plan_request* q, hbx_pipeline_plan* p) {
  if (!q || !p) return HBX_ERR_ARG;
  auto bad = [&](const std::string& m) {
    if (c) return c->fail(HBX_ERR_ARG, m);
    g_noctx_err = m;
    return HBX_ERR_ARG;
  };
  if (q->n_files == 0) return bad("hbx_plan_pipeline: no files");
  if (q->join_lag > 4) return bad("hbx_plan_pipeline: join lag must be 1..4");
  if (q->k3_period > kMaxFresh) return bad("hbx_plan_pipeline: K3 period must be 1..8");
  uint64_t free_b = q->free_bytes;
  if (free_b == 0) {
    if (!c) return bad("hbx_plan_pipeline: free_bytes 0 needs a context");
    std::lock_guard<std::mutex> g(c->mu);
    size_t fr = 0, tot = 0;
    HBX_TRY(c, hipSetDevice(c->device));
    HBX_TRY(c, hipMemGetInfo(&fr, &tot));
    free_b = fr;
  }
  const int64_t lag = q->join_lag > 0 ? q->join_lag : 2;
  const bool host_in = (q->flags & HBX_PLAN_HOST_INPUT) != 0;
  int64_t per = 1;
  if (q->k3_period > 0) {
    per = q->k3_period;
  } else if (q->n_files < 32 && !host_in) {
    // small per-GPU batches: the launch's start-up and tail once per 4 steps
    // (profiles/r05j, r05o: 8 files 2,013 -> 2,056-2,083 GiB/s; 32 files P1
    // 2,277-2,294 vs P2 2,260-2,272)
    per = (q->steps == 0 || q->steps % 4 == 0) ? 4 : (q->steps % 2 == 0) ? 2 : 1;
  }
  // lead (steps an arena stays resident beyond its batch's launches): the join
  // lag at 64 or more files per GPU (round 6: the next batch's K1 follows the
  // launch that finishes the old one through hbx_input_after_oldest; R = 33 at
  // 64 files then holds 31 launches instead of 30: 2,380-2,391 vs 2,303-2,350
  // GiB/s in three alternating pairs, profiles/r06p), lag + 1 below (32 files:
  // 2,229/2,232 vs 2,279/2,273, profiles/r06zf, where the extra chains take
  // CUs from a K1 that already sets the step; 8 files: 2,045 vs 2,082) and for
  // host input
  const int64_t ld = q->lead >= 0 ? q->lead : lag + ((q->n_files >= 64 && !host_in) ? 0 : 1);
  const uint64_t nfull = (std::min<uint64_t>(q->longest_file, HBX_MAX_BLOCK_SIZE) + 8u) >> 6;
  const double frac = q->hbm_frac > 0.0 ? q->hbm_frac : 0.95;
  const uint64_t share = (uint64_t)((double)free_b * frac / (double)std::max<uint32_t>(1u, q->ranks_per_device));
  const uint64_t stride = q->arena_bytes + HBX_PLAN_ARENA_SLACK;
  int64_t r_fit = std::max<int64_t>(ld + 1, (int64_t)(share / stride));
  if (host_in) r_fit = std::min<int64_t>(r_fit, ld + 2);  // PCIe-bound: a shallow pipeline suffices
  auto cdiv = [](uint64_t a, uint64_t b) { return (a + b - 1) / b; };
  auto slice_for = [&](int64_t R) {  // launches of P x B blocks, P submits apart, within R - lead - (P - 1)
    const int64_t launches = std::max<int64_t>(1, (R - ld - per + 1) / per);
    return cdiv(nfull, (uint64_t)(launches * per));
  };
  int64_t R;
  uint64_t B;
  if (q->md5_slice < 0) {
    R = q->arenas > 0 ? q->arenas : r_fit;
    B = slice_for(R);
  } else {
    B = (uint64_t)q->md5_slice;
    R = q->arenas > 0 ? q->arenas
                      : std::min<int64_t>((B == 0 ? 1 : (int64_t)cdiv(nfull, B * per)) * per + ld + per - 1, r_fit);
  }
  const int64_t need = B == 0 ? 1 : (int64_t)cdiv(nfull, B * per);  // K3 launches per batch
  if (need * per + lag + per - 1 > R)
    return bad("hbx_plan_pipeline: pipeline depth " + std::to_string(R) + " < launches per batch " +
               std::to_string(need) + " x period " + std::to_string(per) + " + join lag " + std::to_string(lag) +
               " + " + std::to_string(per - 1) + ": more arenas or a larger slice");
  if (B > 0xFFFFFFFFull || R > 0xFFFFFFFFll) return bad("hbx_plan_pipeline: plan out of range");
  p->resident = (uint32_t)R;
  p->md5_slice = (uint32_t)B;
  p->join_lag = (uint32_t)lag;
  p->lead = (uint32_t)ld;
  p->k3_period = (uint32_t)per;
  p->launches_per_batch = (uint32_t)need;
  p->hbm_bytes = (uint64_t)R * stride;
  return HBX_OK;
}

int hbx_apply_plan(hbx_ctx* c, const hbx_pipeline_plan* p, uint64_t files, uint64_t bytes) {
  if (!c || !p || p->resident == 0) return HBX_ERR_ARG;
  int rc = hbx_set_md5_slice(c, p->md5_slice);
  if (!rc) rc = hbx_set_join_lag(c, p->join_lag);
  if (!rc) rc = hbx_set_k3_period(c, p->k3_period);
  if (!rc) rc = hbx_reserve(c, p->resident + 2u, files, bytes);
  return rc;
}

int hbx_knobs(hbx_ctx* c, char* out, uint64_t cap) {
  if (!c || !out || cap == 0) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  const char* ab = std::getenv("HBX_AB");
  const int n = std::snprintf(
      out, (size_t)cap,
      "{\"ab_env\": %d, \"md5_slice\": %u, \"join_lag\": %u, \"tile_iters\": %u, \"k1_gate\": %u, "
      "\"md5_wgs\": %u, \"plan_mode\": %d, \"k2_own\": %d, \"k4_window\": %u, \"k3_probe\": %d, "
      "\"lean_marks\": %u, \"k3_prod\": %u, \"k3_items\": %u, \"k3_period\": %u, \"meta_kernel\": %u, "
      "\"plan_cut\": %u, \"k1_swz\": %u, \"k3_psets\": %u, \"d2h_kernel\": %u, \"k8_split_streams\": %llu, "
      "\"k8_split_fallbacks\": %llu, \"gate_meta\": %u, \"sdma_warm\": %u, \"sdma_h2d_mask\": %u, "
      "\"sdma_d2h_mask\": %u, \"sdma_warm_ms\": %.3f, \"k3_spin\": %u, \"plan_addr\": %u, \"plan_addr_shift\": %u, \"k1_ext\": %u, \"k1_dma4\": %u, \"k1_early\": %u}",
      (ab && std::atoi(ab) != 0) ? 1 : 0, c->md5_slice, c->join_lag, c->tile_iters, c->k1_gate, c->md5_wgs,
      plan_mode_of(c), c->k2_own, c->k4_window, c->h_probe.p ? 1 : 0, c->lean_marks, c->k3_prod, c->k3_items,
      c->k3_period, c->meta_kernel, c->plan_cut, c->k1_swz, c->k3_psets, c->d2h_kernel,
      (unsigned long long)c->k8_split_streams, (unsigned long long)c->k8_split_fallbacks, c->gate_meta,
      c->sdma_warm, c->sdma_h2d, c->sdma_d2h, c->sdma_warm_ms, c->k3_spin, c->plan_addr, c->plan_addr_shift, c->k1_ext, c->k1_dma4, c->k1_early);
  return (n > 0 && (uint64_t)n < cap) ? HBX_OK : HBX_ERR_ARG;
}

int hbx_set_k3_probe(hbx_ctx* c, int on) {
  if (!c) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  // the launch in flight may still write the records
  if (!c->pending.empty()) return c->fail(HBX_ERR_STATE, "submitted batches are still pending");
  HBX_TRY(c, hipSetDevice(c->device));
  HBX_TRY(c, hipStreamSynchronize(c->hstream));
  if (!on) {
    c->h_probe.release();
    return HBX_OK;
  }
  const size_t n = (size_t)c->md5_wgs * (kK3Threads / 64) * 64;
  HBX_TRY(c, c->h_probe.ensure(n));
  std::memset(c->h_probe.p, 0, n);
  return HBX_OK;
}

int hbx_k3_wave_times(hbx_ctx* c, uint64_t* out, uint32_t max_waves, uint32_t* n_waves) {
  if (!c || !n_waves) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  *n_waves = 0;
  if (!c->h_probe.p) return c->fail(HBX_ERR_STATE, "K3 probe not enabled (hbx_set_k3_probe)");
  HBX_TRY(c, hipSetDevice(c->device));
  HBX_TRY(c, hipStreamSynchronize(c->hstream));
  const uint32_t n = c->md5_wgs * (kK3Threads / 64);
  if (out) std::memcpy(out, c->h_probe.p, (size_t)std::min(n, max_waves) * 64);
  *n_waves = n;
  return HBX_OK;
}

int hbx_stage_times(hbx_ctx* c, float ms[5]) {
  if (!c || !ms) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  for (int i = 0; i < 5; i++) ms[i] = c->stage_ms[i];
  return HBX_OK;
}

int hbx_set_md5_slice(hbx_ctx* c, uint32_t blocks) {
  if (!c) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  // a pending batch's launch count was fixed at submit from the slice of
  // that moment: changing it now would finalize batches whose chains are
  // not all hashed
  if (!c->pending.empty()) return c->fail(HBX_ERR_STATE, "submitted batches are still pending");
  c->md5_slice = blocks;
  return HBX_OK;
}

int hbx_reserve(hbx_ctx* c, uint32_t batches, uint64_t files, uint64_t bytes) {
  if (!c || files > 0xFFFFFFFFull) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  return reserve_locked(c, batches, files, bytes);
}

int reserve_locked(hbx_ctx* c, uint32_t batches, uint64_t files, uint64_t bytes) {
  if (!c->pending.empty()) return c->fail(HBX_ERR_STATE, "submitted batches are still pending");
  HBX_TRY(c, hipSetDevice(c->device));
  const uint64_t caps = bytes / HBX_MIN_BLOCK_SIZE + files;  // >= sum of max_chunks over the files
  const uint64_t tiles = bytes / ((uint64_t)(c->tile_iters ? c->tile_iters : kTileItersMin) * HBX_MIN_BLOCK_SIZE) + files;
  const uint64_t slices = bytes / kSlice + files;
  const size_t meta_bytes = files * 8 * 4 + tiles * sizeof(uint4);
  int rc = HBX_OK;
  for (int t = 0; t < 2 && !rc; t++) rc = ensure_shared(c, c->d_ssum[t], (slices + 1) * sizeof(uint2));
  if (!rc) rc = ensure_shared(c, c->d_plan, 2 * kPlanBins * sizeof(uint32_t));
  for (int t = 0; t < 3 && !rc; t++) {
    rc = ensure_shared(c, c->d_order[t], ((uint64_t)batches * caps + 64) * sizeof(OrderEntry));
    if (!rc) rc = ensure_shared(c, c->d_octl[t], 256);
    if (!rc) rc = ensure_shared(c, c->d_q[t], (((uint64_t)batches * caps + 64) / 64 + 2) * 8 * 8);
  }
  if (rc) return rc;
  std::vector<Batch*> ready;
  while (ready.size() < batches) {
    Batch* b = acquire_batch(c);  // pooled first, then new
    if (!b) break;
    ready.push_back(b);
    const size_t rbytes = res_layout(files, caps).total;
    for (auto r : {b->h_meta.ensure(meta_bytes), b->d_meta.ensure(meta_bytes), b->d_res.ensure(rbytes),
                   b->d_run.ensure(caps * sizeof(Chain)), b->d_fresh.ensure(caps * sizeof(OrderEntry)),
                   b->d_fcnt.ensure(256), b->h_res.ensure(rbytes)})
      if (r != hipSuccess && !rc) rc = c->hip(r, "hbx_reserve");
    if (rc) break;
  }
  for (Batch* b : ready) c->pool.push_back(b);
  if (!rc && ready.size() < batches) rc = c->fail(HBX_ERR_HIP, "cannot create batch events");
  return rc;
}

int hbx_stage_totals(hbx_ctx* c, double ms[5], uint64_t launches[5], int reset) {
  if (!c) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  harvest_timings(c);
  if (c->hstream && hipStreamQuery(c->hstream) == hipSuccess) c->k3_done_upto = c->launches;
  harvest_k3(c);
  for (int i = 0; i < 5; i++) {
    if (ms) ms[i] = c->tot_ms[i];
    if (launches) launches[i] = c->tot_n[i];
    if (reset) {
      c->tot_ms[i] = 0.0;
      c->tot_n[i] = 0;
    }
  }
  return HBX_OK;
}

int hbx_chunk_hash_device(hbx_ctx* c, const void* d_arena, uint64_t n, const uint64_t* offs,
                          const uint64_t* lens, uint64_t* cut_ends, uint8_t* ids,
                          const uint64_t* out_base, const uint64_t* caps,
                          hbx_file_summary* sums) {
  if (!c) return HBX_ERR_ARG;
  if (n && (!d_arena || !offs || !lens || !out_base || !caps)) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->pending.empty()) return c->fail(HBX_ERR_STATE, "submitted batches are still pending");
  HBX_TRY(c, hipSetDevice(c->device));
  return run_device_sync(c, d_arena, n, offs, lens, cut_ends, ids, out_base, caps, sums);
}

int hbx_submit_device(hbx_ctx* c, const void* d_arena, uint64_t n, const uint64_t* offs,
                      const uint64_t* lens, uint64_t* cut_ends, uint8_t* ids,
                      const uint64_t* out_base, const uint64_t* caps, hbx_file_summary* sums) {
  if (!c) return HBX_ERR_ARG;
  if (n && (!d_arena || !offs || !lens || !out_base || !caps)) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HBX_TRY(c, hipSetDevice(c->device));
  return submit_batch(c, d_arena, n, offs, lens, cut_ends, ids, out_base, caps, sums,
                      c->md5_slice ? c->md5_slice : kBudgetAll);
}

int hbx_wait(hbx_ctx* c) {
  if (!c) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HBX_TRY(c, hipSetDevice(c->device));
  return wait_oldest(c);
}

int hbx_pending(hbx_ctx* c) {
  if (!c) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  return (int)c->pending.size();
}

int hbx_chunk_hash_batch(hbx_ctx* c, uint64_t n, const uint8_t* const* datas,
                         const uint64_t* lens, uint64_t* cut_ends, uint8_t* ids,
                         const uint64_t* out_base, const uint64_t* caps,
                         hbx_file_summary* sums) {
  if (!c) return HBX_ERR_ARG;
  if (n && (!datas || !lens || !out_base || !caps)) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->pending.empty()) return c->fail(HBX_ERR_STATE, "submitted batches are still pending");
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
  hbx_file_summary s{};
  int rc = hbx_chunk_hash_batch(c, 1, &data, &len, cut_ends, ids, &base, &cap, &s);
  // the count is meaningful on success and on HBX_ERR_CAPACITY (the caller
  // retries with that many slots); otherwise it is left untouched
  if (n_chunks && (rc == HBX_OK || rc == HBX_ERR_CAPACITY)) *n_chunks = s.n_chunks;
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

// MD5(data) on the device (K5 over the raw message): core.Hash (core.go:46-48),
// the primitive under Hmac/DeepHmac (core.go:51-80), whose KAT rows
// (core_test.go:23-30) tests/test_gpu_parity.py runs through this call.
int hbx_md5(hbx_ctx* c, const uint8_t* data, uint64_t len, uint8_t out[16]) {
  if (!c || !out || (len && !data) || len > 0xFFFFFFFEull - 16ull) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HBX_TRY(c, hipSetDevice(c->device));
  HBX_TRY(c, c->d_msg.ensure(len + 16));
  uint8_t* dm = c->d_msg.as<uint8_t>();
  if (len) HBX_TRY(c, hipMemcpyAsync(dm + 16, data, len, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(hbx_k5_md5_raw, dim3(1), dim3(64), 0, c->stream, dm + 16, (uint32_t)len,
                     reinterpret_cast<uint32_t*>(dm));
  HBX_TRY(c, hipGetLastError());
  HBX_TRY(c, hipMemcpyAsync(out, dm, 16, hipMemcpyDeviceToHost, c->stream));
  HBX_TRY(c, hipStreamSynchronize(c->stream));
  return HBX_OK;
}

namespace {
// K6 over n blocks whose data is already on the device (block i at
// arena + offs[i]); lanes are ordered longest first so each wave's 64 chains
// are about equally long.
int verify_device(hbx_ctx* c, const uint8_t* arena, uint64_t n, const uint64_t* offs,
                  const uint64_t* lens, const uint8_t* links, const uint64_t* link_base,
                  const uint32_t* n_links, uint8_t* ids, const uint8_t* expect, uint8_t* ok,
                  uint64_t* n_bad) {
  if (n_bad) *n_bad = 0;
  if (n == 0) return HBX_OK;
  if (n > 0xFFFFFFFFull) return c->fail(HBX_ERR_ARG, "too many blocks");
  uint64_t nlinks_total = 0;
  for (uint64_t i = 0; i < n; i++) {
    const uint32_t nl = n_links ? n_links[i] : 0u;
    if (nl && (!links || !link_base)) return c->fail(HBX_ERR_ARG, "links missing");
    if (lens[i] + 8ull + 16ull * nl + 128ull > 0xFFFFFFFFull) return c->fail(HBX_ERR_ARG, "block too large");
    if (nl) nlinks_total = std::max(nlinks_total, link_base[i] + nl);
  }
  std::vector<uint32_t> perm(n);
  for (uint64_t i = 0; i < n; i++) perm[i] = (uint32_t)i;
  std::stable_sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t b) { return lens[a] > lens[b]; });
  HBX_TRY(c, c->d_vdesc.ensure(n * sizeof(VerifyDesc)));
  HBX_TRY(c, c->d_vlinks.ensure(std::max<uint64_t>(16 * nlinks_total, 16)));
  HBX_TRY(c, c->d_vout.ensure(n * 17));
  HBX_TRY(c, c->d_zeros.ensure(256));
  if (expect) HBX_TRY(c, c->d_vexp.ensure(n * 16));
  const uint8_t* dl = c->d_vlinks.as<uint8_t>();
  std::vector<VerifyDesc> desc(n);
  std::vector<uint8_t> exp_p(expect ? n * 16 : 0);
  for (uint64_t k = 0; k < n; k++) {
    const uint32_t i = perm[k];
    const uint32_t nl = n_links ? n_links[i] : 0u;
    desc[k].src = reinterpret_cast<uint64_t>(arena + offs[i]);
    desc[k].links = reinterpret_cast<uint64_t>(dl + (nl ? 16 * link_base[i] : 0));
    desc[k].len = (uint32_t)lens[i];
    desc[k].n_links = nl;
    desc[k].pad = 0;
    if (expect) std::memcpy(&exp_p[16 * k], expect + 16ull * i, 16);
  }
  hipStream_t s = c->stream;
  HBX_TRY(c, hipMemsetAsync(c->d_zeros.p, 0, 256, s));
  HBX_TRY(c, hipMemcpyAsync(c->d_vdesc.p, desc.data(), n * sizeof(VerifyDesc), hipMemcpyHostToDevice, s));
  if (nlinks_total) HBX_TRY(c, hipMemcpyAsync(c->d_vlinks.p, links, 16 * nlinks_total, hipMemcpyHostToDevice, s));
  if (expect) HBX_TRY(c, hipMemcpyAsync(c->d_vexp.p, exp_p.data(), n * 16, hipMemcpyHostToDevice, s));
  uint8_t* dout = c->d_vout.as<uint8_t>();
  hipLaunchKernelGGL(hbx_k6_hash_blocks, dim3((uint32_t)((n + 63) / 64)), dim3(64), 0, s,
                     c->d_vdesc.as<VerifyDesc>(), (uint32_t)n, c->d_zeros.as<uint8_t>(),
                     reinterpret_cast<uint32_t*>(dout), expect ? c->d_vexp.as<uint32_t>() : nullptr,
                     dout + 16 * n);
  HBX_TRY(c, hipGetLastError());
  std::vector<uint8_t> out(n * 17);
  HBX_TRY(c, hipMemcpyAsync(out.data(), dout, n * 17, hipMemcpyDeviceToHost, s));
  HBX_TRY(c, hipStreamSynchronize(s));
  uint64_t bad = 0;
  for (uint64_t k = 0; k < n; k++) {
    const uint32_t i = perm[k];
    if (ids) std::memcpy(ids + 16ull * i, &out[16 * k], 16);
    if (expect) {
      const uint8_t good = out[16 * n + k];
      if (ok) ok[i] = good;
      bad += good ? 0 : 1;
    }
  }
  if (n_bad) *n_bad = bad;
  return HBX_OK;
}
}  // namespace

int hbx_verify_blocks_device(hbx_ctx* c, const void* d_arena, uint64_t n, const uint64_t* offs,
                             const uint64_t* lens, const uint8_t* links, const uint64_t* link_base,
                             const uint32_t* n_links, uint8_t* ids, const uint8_t* expect, uint8_t* ok,
                             uint64_t* n_bad) {
  if (!c || (n && (!d_arena || !offs || !lens))) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->pending.empty()) return c->fail(HBX_ERR_STATE, "submitted batches are still pending");
  HBX_TRY(c, hipSetDevice(c->device));
  return verify_device(c, static_cast<const uint8_t*>(d_arena), n, offs, lens, links, link_base, n_links,
                       ids, expect, ok, n_bad);
}

int hbx_verify_blocks(hbx_ctx* c, uint64_t n, const uint8_t* const* datas, const uint64_t* lens,
                      const uint8_t* links, const uint64_t* link_base, const uint32_t* n_links,
                      uint8_t* ids, const uint8_t* expect, uint8_t* ok, uint64_t* n_bad) {
  if (!c || (n && (!datas || !lens))) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->pending.empty()) return c->fail(HBX_ERR_STATE, "submitted batches are still pending");
  HBX_TRY(c, hipSetDevice(c->device));
  std::vector<uint64_t> offs(n);
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; i++) {
    if (lens[i] && !datas[i]) return c->fail(HBX_ERR_ARG, "null block data");
    offs[i] = total;
    total += (lens[i] + 255) & ~uint64_t(255);
  }
  HBX_TRY(c, c->d_stage.ensure(total + 65536));
  uint8_t* arena = c->d_stage.as<uint8_t>();
  for (uint64_t i = 0; i < n; i++)
    if (lens[i]) HBX_TRY(c, hipMemcpyAsync(arena + offs[i], datas[i], lens[i], hipMemcpyHostToDevice, c->stream));
  return verify_device(c, arena, n, offs.data(), lens, links, link_base, n_links, ids, expect, ok, n_bad);
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
  if (int frc = flush_input_wait(c)) return frc;
  HBX_TRY(c, hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, c->stream));
  HBX_TRY(c, hipStreamSynchronize(c->stream));
  return HBX_OK;
}

// ---- files on disk -> pinned -> HBM -> results (BASELINE configs[4]) ----
namespace {

// Read whole files into dst + offs[i] with `threads` threads (files are
// independent).  Returns 0 or HBX_ERR_IO with the offending path in err.
// With `status` (per file of this list), the failures the reference treats
// per file are recorded there instead of failing the call, and the file is
// skipped (hbx_store_paths_status): an open() failure (os.Open returns it,
// storeDir logs and continues: store.go:101-103, 221-224) and a read failing
// with EBADF (minorPathError, hashback_unix.go:57-63).  Any other read error
// or a short file is a panic in storeFile (CopyNOrPanic, utils.go:95-99):
// the call fails either way.
int read_files(uint64_t n, const char* const* paths, const uint64_t* lens, const uint64_t* offs,
               uint8_t* dst, uint32_t threads, std::string& err, int32_t* status = nullptr) {
  std::atomic<uint64_t> next{0};
  std::atomic<int> failed{0};
  std::mutex emu;
  auto worker = [&]() {
    for (;;) {
      const uint64_t i = next.fetch_add(1);
      if (i >= n || failed.load()) return;
      if (status) status[i] = 0;
      const int fd = ::open(paths[i], O_RDONLY | O_CLOEXEC);
      int e = fd < 0 ? errno : 0;
      if (fd < 0 && status) {
        status[i] = e ? e : EIO;
        continue;
      }
      uint64_t got = 0;
      while (fd >= 0 && got < lens[i]) {
        const ssize_t r = ::pread(fd, dst + offs[i] + got, lens[i] - got, (off_t)got);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) {
          e = r < 0 ? errno : 0;  // 0: end of file before lens[i] bytes
          break;
        }
        got += (uint64_t)r;
      }
      if (fd >= 0) ::close(fd);
      if (fd >= 0 && got == lens[i]) continue;
      if (status && e == EBADF) {
        status[i] = EBADF;
        continue;
      }
      failed.store(1);
      std::lock_guard<std::mutex> g(emu);
      err = std::string("cannot read ") + std::to_string(lens[i]) + " bytes of " + paths[i] + ": " +
            (fd < 0 ? std::string("open: ") + std::strerror(e)
                    : e ? std::string(std::strerror(e)) : "end of file after " + std::to_string(got) + " bytes");
      return;
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

namespace {
int deflate_device(hbx_ctx* c, uint64_t n, const uint64_t* src, const uint64_t* lens, const uint64_t* dst,
                   uint64_t* out_lens);

// Output of hbx_store_paths_z (null members: no compression).
struct ZOut {
  uint8_t* zout = nullptr;
  const uint64_t* zbase = nullptr;
  uint64_t* zoff = nullptr;
  uint64_t* zlen = nullptr;
  hbx_batch_ready_fn ready = nullptr;  // called once a batch's results are all written
  void* user = nullptr;
};
// A collected batch whose device arena still holds its files.
struct ZJob {
  uint64_t first = 0, count = 0;
  const uint8_t* arena = nullptr;
  std::vector<uint64_t> offs;
};

// CompressData of every chunk of a collected batch (client.go:249-258),
// asynchronous: K7 reads the batch's arena on the engine's compression
// streams (one per stage) and the streams come back in one D2H copy into a pinned stage, while
// the caller's loop goes on reading and copying later batches.  Two stages
// rotate; a stage is unpacked (streams placed per file at zout[zbase[f] ..],
// the batch's callback) before it is reused, and every job is unpacked in
// FIFO order before hbx_store_paths_z returns.
struct ZPend {
  ZJob job;
  int stage = 0;
  std::vector<uint64_t> dst;  // stream offset of each chunk in the stage
  std::shared_future<int> fin;  // its unpack (z_finish), on a worker thread
  double t_sync = 0.0;          // HBX_ZDIAG: time that unpack waited for the GPU
  std::string err;              // the worker's error text: it never writes c->err,
                                // which the main loop owns; zdrain_one copies it
};

int z_start(hbx_ctx* c, ZPend& zp, const uint64_t* cut_ends, const uint64_t* out_base,
            const hbx_file_summary* sums) {
  auto& Z = c->zs[zp.stage];
  std::vector<hbxz::ZBlock> zb;
  uint64_t d = 0, nseg = 0;
  for (uint64_t i = 0; i < zp.job.count; i++) {
    const uint64_t f = zp.job.first + i;
    uint64_t start = 0;
    for (uint32_t q = 0; q < sums[f].n_chunks; q++) {
      const uint64_t e = cut_ends[out_base[f] + q];
      const uint64_t len = e - start, ns = (len + hbxz::kSeg - 1) / hbxz::kSeg;
      zb.push_back(hbxz::ZBlock{reinterpret_cast<uint64_t>(zp.job.arena + zp.job.offs[i] + start), d, len,
                                (uint32_t)nseg, (uint32_t)ns});
      zp.dst.push_back(d);
      d += (hbx_deflate_bound(len) + 15) & ~uint64_t(15);
      nseg += ns;
      start = e;
    }
  }
  const uint64_t n = zb.size();
  if (n == 0) return HBX_OK;
  if (nseg > 0x7FFFFFFFull) return c->fail(HBX_ERR_ARG, "too much data in one batch");
  if (!Z.stream) HBX_TRY(c, hipStreamCreateWithFlags(&Z.stream, hipStreamNonBlocking));
  if (!Z.done) HBX_TRY(c, hipEventCreateWithFlags(&Z.done, hipEventDisableTiming));
  HBX_TRY(c, Z.out.ensure(d + 64));
  HBX_TRY(c, Z.stage.ensure(d + 64));
  HBX_TRY(c, Z.desc.ensure(n * sizeof(hbxz::ZBlock)));
  HBX_TRY(c, Z.lens.ensure(n * 8));
  HBX_TRY(c, Z.blk.ensure(n * sizeof(hbxz::ZBlock)));
  HBX_TRY(c, Z.info.ensure(std::max<uint64_t>(nseg, 1) * sizeof(hbxz::SegInfo)));
  HBX_TRY(c, Z.off.ensure(std::max<uint64_t>(nseg, 1) * 8));
  HBX_TRY(c, Z.len.ensure(n * 8));
  HBX_TRY(c, Z.img.ensure(std::max<uint64_t>(nseg, 1) * hbxz::kSlot));
  const uint64_t base = reinterpret_cast<uint64_t>(Z.out.p);
  for (auto& x : zb) x.dst += base;  // stage offsets -> device addresses
  std::memcpy(Z.desc.p, zb.data(), n * sizeof(hbxz::ZBlock));
  hipStream_t s = Z.stream;
  HBX_TRY(c, hipMemcpyAsync(Z.blk.p, Z.desc.p, n * sizeof(hbxz::ZBlock), hipMemcpyHostToDevice, s));
  const hbxz::ZBlock* dz = Z.blk.as<hbxz::ZBlock>();
  hipLaunchKernelGGL(hbx_k7_deflate_entropy, dim3((uint32_t)nseg), dim3(hbxz::kEThreads), 0, s, dz, (uint32_t)n,
                     (uint32_t)nseg, Z.info.as<hbxz::SegInfo>());
  hipLaunchKernelGGL(hbx_k7_deflate_size, dim3((uint32_t)nseg), dim3(hbxz::kThreads), 0, s, dz, (uint32_t)n,
                     (uint32_t)nseg, Z.info.as<hbxz::SegInfo>(), Z.img.as<uint32_t>());
  hipLaunchKernelGGL(hbx_k7_deflate_code, dim3((uint32_t)nseg), dim3(hbxz::kThreads), 0, s, dz, (uint32_t)n,
                     (uint32_t)nseg, Z.info.as<hbxz::SegInfo>(), Z.img.as<uint32_t>());
  HBX_TRY(c, hipGetLastError());
  hipLaunchKernelGGL(hbx_k7_deflate_plan, dim3((uint32_t)n), dim3(64), 0, s, dz, (uint32_t)n,
                     Z.info.as<hbxz::SegInfo>(), Z.off.as<uint64_t>(), Z.len.as<uint64_t>());
  HBX_TRY(c, hipGetLastError());
  hipLaunchKernelGGL(hbx_k7_deflate_write, dim3((uint32_t)nseg), dim3(hbxz::kWThreads), 0, s, (uint32_t)nseg,
                     Z.info.as<hbxz::SegInfo>(), Z.img.as<uint32_t>(), Z.off.as<uint64_t>(), dz, (uint32_t)n);
  HBX_TRY(c, hipGetLastError());
  HBX_TRY(c, hipMemcpyAsync(Z.lens.p, Z.len.p, n * 8, hipMemcpyDeviceToHost, s));
  HBX_TRY(c, hipMemcpyAsync(Z.stage.p, Z.out.p, d, hipMemcpyDeviceToHost, s));
  HBX_TRY(c, hipEventRecord(Z.done, s));
  return HBX_OK;
}

// Wait for a started job, place its streams and call the batch back.
// Runs on a worker thread: reports errors only through zp.err (never c->err,
// c->hip or c->fail, which the caller's thread uses meanwhile).
int z_finish(const hbx_ctx* c, ZPend& zp, const uint64_t* out_base, const hbx_file_summary* sums, const ZOut& z,
             uint32_t threads, double& t_sync) {
  const auto& Z = c->zs[zp.stage];
  const uint64_t nc = zp.dst.size();
  if (nc) {
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t e = hipEventSynchronize(Z.done);
    if (e != hipSuccess) {
      zp.err = std::string("hipEventSynchronize(compression stage): ") + hipGetErrorString(e);
      return HBX_ERR_HIP;
    }
    t_sync += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const uint8_t* h = Z.stage.as<uint8_t>();
    const uint64_t* ol = Z.lens.as<uint64_t>();
    // placement (serial, cheap), then the copies out of the pinned stage on
    // `threads` threads (one thread copies a few GB/s)
    std::vector<uint64_t> to(nc);
    uint64_t k = 0;
    for (uint64_t i = 0; i < zp.job.count; i++) {
      const uint64_t f = zp.job.first + i;
      uint64_t run = z.zbase[f];
      for (uint32_t q = 0; q < sums[f].n_chunks; q++, k++) {
        to[k] = run;
        z.zoff[out_base[f] + q] = run;
        z.zlen[out_base[f] + q] = ol[k];
        run += ol[k];
      }
    }
    const uint32_t nt = std::max<uint32_t>(1u, std::min<uint32_t>(threads, 64u));
    std::vector<std::thread> pool;
    for (uint32_t t = 0; t < nt; t++)
      pool.emplace_back([&, t] {
        for (uint64_t i = t; i < nc; i += nt) std::memcpy(z.zout + to[i], h + zp.dst[i], ol[i]);
      });
    for (auto& th : pool) th.join();
  }
  if (z.ready) z.ready(z.user, zp.job.first, zp.job.count);
  return HBX_OK;
}

int store_paths_impl(hbx_ctx* c, uint64_t n, const char* const* paths, const uint64_t* lens,
                     uint64_t* cut_ends, uint8_t* ids, const uint64_t* out_base, const uint64_t* caps,
                     hbx_file_summary* sums, uint32_t io_threads, uint64_t batch_bytes, const ZOut& z,
                     int32_t* status = nullptr);
}  // namespace

int hbx_store_paths(hbx_ctx* c, uint64_t n, const char* const* paths, const uint64_t* lens,
                    uint64_t* cut_ends, uint8_t* ids, const uint64_t* out_base,
                    const uint64_t* caps, hbx_file_summary* sums, uint32_t io_threads,
                    uint64_t batch_bytes) {
  if (!c) return HBX_ERR_ARG;
  if (n && (!paths || !lens || !out_base || !caps)) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  return store_paths_impl(c, n, paths, lens, cut_ends, ids, out_base, caps, sums, io_threads, batch_bytes,
                          ZOut{});
}

int hbx_store_paths_status(hbx_ctx* c, uint64_t n, const char* const* paths, const uint64_t* lens,
                           uint64_t* cut_ends, uint8_t* ids, const uint64_t* out_base, const uint64_t* caps,
                           hbx_file_summary* sums, int32_t* status, uint32_t io_threads, uint64_t batch_bytes,
                           uint8_t* zout, const uint64_t* zbase, uint64_t* zoff, uint64_t* zlen,
                           hbx_batch_ready_fn ready, void* user) {
  if (!c) return HBX_ERR_ARG;
  const bool z = zout || zbase || zoff || zlen;
  if (n && (!paths || !lens || !out_base || !caps || !status)) return HBX_ERR_ARG;
  if (n && z && (!sums || !zout || !zbase || !zoff || !zlen)) return HBX_ERR_ARG;
  if (!z && ready) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  for (uint64_t i = 0; i < n; i++) status[i] = 0;
  return store_paths_impl(c, n, paths, lens, cut_ends, ids, out_base, caps, sums, io_threads, batch_bytes,
                          z ? ZOut{zout, zbase, zoff, zlen, ready, user} : ZOut{}, status);
}

uint64_t hbx_deflate_file_bound(uint64_t len) {
  return len + 16ull * hbx_max_chunks(len) + 5ull * (len / hbxz::kSeg);
}

int hbx_store_paths_z(hbx_ctx* c, uint64_t n, const char* const* paths, const uint64_t* lens,
                      uint64_t* cut_ends, uint8_t* ids, const uint64_t* out_base, const uint64_t* caps,
                      hbx_file_summary* sums, uint32_t io_threads, uint64_t batch_bytes, uint8_t* zout,
                      const uint64_t* zbase, uint64_t* zoff, uint64_t* zlen) {
  if (!c) return HBX_ERR_ARG;
  if (n && (!paths || !lens || !out_base || !caps || !sums || !zout || !zbase || !zoff || !zlen))
    return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  return store_paths_impl(c, n, paths, lens, cut_ends, ids, out_base, caps, sums, io_threads, batch_bytes,
                          ZOut{zout, zbase, zoff, zlen, nullptr, nullptr});
}

int hbx_store_paths_zcb(hbx_ctx* c, uint64_t n, const char* const* paths, const uint64_t* lens,
                        uint64_t* cut_ends, uint8_t* ids, const uint64_t* out_base, const uint64_t* caps,
                        hbx_file_summary* sums, uint32_t io_threads, uint64_t batch_bytes, uint8_t* zout,
                        const uint64_t* zbase, uint64_t* zoff, uint64_t* zlen, hbx_batch_ready_fn ready,
                        void* user) {
  if (!c) return HBX_ERR_ARG;
  if (n && (!paths || !lens || !out_base || !caps || !sums || !zout || !zbase || !zoff || !zlen))
    return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  return store_paths_impl(c, n, paths, lens, cut_ends, ids, out_base, caps, sums, io_threads, batch_bytes,
                          ZOut{zout, zbase, zoff, zlen, ready, user});
}

namespace {
int store_paths_impl(hbx_ctx* c, uint64_t n, const char* const* paths, const uint64_t* lens,
                     uint64_t* cut_ends, uint8_t* ids, const uint64_t* out_base, const uint64_t* caps,
                     hbx_file_summary* sums, uint32_t io_threads, uint64_t batch_bytes, const ZOut& z,
                     int32_t* status) {
  if (!c->pending.empty()) return c->fail(HBX_ERR_STATE, "submitted batches are still pending");
  HBX_TRY(c, hipSetDevice(c->device));
  if (batch_bytes < (64ull << 20)) batch_bytes = 64ull << 20;
  for (hipEvent_t& e : c->h2d_done)
    if (!e) HBX_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  // Pipeline: files of batch k are read (io_threads) into pinned slot k % 2
  // while earlier batches copy and hash; the H2D copy runs on the scan
  // stream into device arena k % depth, and the batch joins the time-sliced
  // MD5 chains.  A pinned slot is free once its copy has completed, a device
  // arena once its batch has been collected.
  const uint32_t budget = c->md5_slice ? c->md5_slice : kBudgetAll;
  const uint64_t nfull_max = (HBX_MAX_BLOCK_SIZE + 8ull) >> 6;
  // a batch's chains join the launch join_lag submits later (up to P - 1
  // more with a K3 period P) and need ceil(nfull / (P x budget)) launches P
  // submits apart, so this many arenas keep the collect from forcing a drain
  const uint64_t lb = launch_budget(c, budget), per = std::max<uint32_t>(1, c->k3_period);
  const size_t depth = budget == kBudgetAll ? 2 : (size_t)std::min<uint64_t>(
      64, (nfull_max + lb - 1) / lb * per + c->join_lag + per);
  if (c->d_ring.size() < depth) c->d_ring.resize(depth);
  // size every staging buffer once, for the largest batch this call forms
  // (growing one later would re-pin host memory or drain the streams)
  uint64_t biggest = 0, zbytes = 0, zchunks = 0, zsegs = 0, most_files = 0;
  for (uint64_t i = 0; i < n;) {
    uint64_t tot = 0, cnt = 0;
    while (i < n && (cnt == 0 || tot + lens[i] <= batch_bytes) && cnt < 65536) {
      tot += (lens[i] + 255) & ~uint64_t(255);
      i++;
      cnt++;
    }
    biggest = std::max(biggest, tot);
    most_files = std::max(most_files, cnt);
    // compression stage bounds of this batch: chunks <= a file's
    // max_chunks, a chunk's stream <= hbx_deflate_bound rounded to 16 B
    const uint64_t nch = tot / HBX_MIN_BLOCK_SIZE + cnt;
    zchunks = std::max(zchunks, nch);
    zsegs = std::max(zsegs, tot / hbxz::kSeg + nch);
    zbytes = std::max<uint64_t>(zbytes, tot + 5ull * (tot / hbxz::kSeg) + 31ull * nch + 64);
  }
  for (PinBuf& h : c->h_read) HBX_TRY(c, h.ensure(biggest + 65536));
  if (z.zout)  // every compression stage sized once (growing one would re-pin or drain the device)
    for (auto& Z : c->zs) {
      HBX_TRY(c, Z.out.ensure(zbytes));
      HBX_TRY(c, Z.stage.ensure(zbytes));
      HBX_TRY(c, Z.desc.ensure(zchunks * sizeof(hbxz::ZBlock)));
      HBX_TRY(c, Z.lens.ensure(zchunks * 8));
      HBX_TRY(c, Z.blk.ensure(zchunks * sizeof(hbxz::ZBlock)));
      HBX_TRY(c, Z.info.ensure(std::max<uint64_t>(zsegs, 1) * sizeof(hbxz::SegInfo)));
      HBX_TRY(c, Z.off.ensure(std::max<uint64_t>(zsegs, 1) * 8));
      HBX_TRY(c, Z.len.ensure(zchunks * 8));
      HBX_TRY(c, Z.img.ensure(std::max<uint64_t>(zsegs, 1) * hbxz::kSlot));
    }
  for (size_t i = 0; i < depth; i++) {
    int r0 = ensure_shared(c, c->d_ring[i], biggest + 65536);
    if (r0) return r0;
  }
  // every batch slot of the pipeline sized for the largest batch up front: a
  // pooled batch that met a larger batch later reallocated its pinned meta and
  // result buffers inside that submit (19-28 ms per submit of config 5,
  // HBX_TRACE_SLOW_SUBMIT "buffers", profiles/r06e)
  if (int r0 = reserve_locked(c, (uint32_t)depth + 2u, most_files, biggest)) return r0;
  auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  bool slot_used[2] = {false, false};
  std::vector<uint64_t> offs, skip_lens;
  uint64_t f = 0, k = 0;
  int rc = HBX_OK;
  // with compression, each collected batch is compressed from its arena on
  // the compression stream (z_start); the next batch copied into that arena
  // waits for it on the GPU, and the host unpacks a stage (z_finish, FIFO)
  // before reusing it and at the end
  std::deque<ZJob> jobs;
  std::deque<ZPend> zq;
  uint64_t zjobs = 0;
  double zt[4] = {0, 0, 0, 0};  // HBX_ZDIAG: wait_oldest | z_start | z_finish | its event waits
  int arena_zstage = -1;  // the stage that reads the arena just freed by collect()
  auto zdrain_one = [&]() -> int {
    const double t0 = now();
    const int r = zq.front().fin.get();
    if (r && !zq.front().err.empty()) c->err = zq.front().err;  // the worker's text, on this thread
    zt[2] += now() - t0;
    zt[3] += zq.front().t_sync;
    zq.pop_front();
    return r;
  };
  // every compression stream idle: K7 of a failed job may still read an arena
  // that the next call rewrites
  auto zsync_all = [&]() {
    for (auto& Z : c->zs)
      if (Z.stream) (void)hipStreamSynchronize(Z.stream);
  };
  auto collect = [&]() -> int {
    const double t0 = now();
    int r = wait_oldest(c);
    zt[0] += now() - t0;
    arena_zstage = -1;
    if (z.zout && !jobs.empty()) {
      if (!r && zq.size() >= (size_t)hbx_ctx::kZStages) r = zdrain_one();  // the stage this job takes
      if (!r) {
        ZPend zp;
        zp.job = std::move(jobs.front());
        zp.stage = (int)(zjobs++ % (uint64_t)hbx_ctx::kZStages);
        const double t1 = now();
        r = z_start(c, zp, cut_ends, out_base, sums);
        zt[1] += now() - t1;
        arena_zstage = zp.stage;
        // the unpack runs on a worker thread while this loop reads and copies
        // the next batches; each waits for its predecessor (FIFO callbacks)
        std::shared_future<int> prev = zq.empty() ? std::shared_future<int>() : zq.back().fin;
        zq.push_back(std::move(zp));
        if (!r) {
          ZPend* zpp = &zq.back();  // a deque keeps element addresses on push_back / pop_front
          const uint32_t ut = std::max<uint32_t>(1u, io_threads / 2u);
          zpp->fin = std::async(std::launch::async, [c, zpp, prev, out_base, sums, &z, ut]() -> int {
                       if (prev.valid()) {
                         const int r0 = prev.get();
                         if (r0) return r0;
                       }
                       (void)hipSetDevice(c->device);
                       return z_finish(c, *zpp, out_base, sums, z, ut, zpp->t_sync);
                     }).share();
        } else {
          std::promise<int> pr;
          pr.set_value(r);
          zq.back().fin = pr.get_future().share();
        }
      }
      jobs.pop_front();
    }
    return r;
  };
  while (f < n && rc == HBX_OK) {
    const uint64_t first = f;
    offs.clear();
    uint64_t tot = 0;
    while (f < n && (offs.empty() || tot + lens[f] <= batch_bytes) && offs.size() < 65536) {
      offs.push_back(tot);
      tot += (lens[f] + 255) & ~uint64_t(255);
      f++;
    }
    const int p = (int)(k & 1);
    DevBuf& arena = c->d_ring[k % depth];
    double t0 = now();
    if (c->pending.size() >= depth && (rc = collect())) break;  // frees arena k % depth
    double t1 = now();
    if (slot_used[p] && (rc = c->hip(hipEventSynchronize(c->h2d_done[p]), "h2d wait"))) break;
    double t2 = now();
    rc = read_files(f - first, paths + first, lens + first, offs.data(), c->h_read[p].as<uint8_t>(),
                    io_threads, c->err, status ? status + first : nullptr);
    c->io_s[0] += now() - t2;
    c->io_s[1] += t1 - t0;
    c->io_s[2] += t2 - t1;
    if (rc) break;
    // the arena's previous batch may still be read by its compression job
    if (arena_zstage >= 0 && c->zs[arena_zstage].done &&
        (rc = c->hip(hipStreamWaitEvent(c->stream, c->zs[arena_zstage].done, 0), "hipStreamWaitEvent")))
      break;
    arena_zstage = -1;
    const auto tc = std::chrono::steady_clock::now();
    if ((rc = c->hip(hipMemcpyAsync(arena.p, c->h_read[p].p, tot, hipMemcpyHostToDevice, c->stream),
                     "hipMemcpyAsync")))
      break;
    c->max_copy_ms = std::max(c->max_copy_ms, ms_since(tc));
    g_slow.call("store_paths h2d: hipMemcpyAsync", tc, c->launches);
    if ((rc = c->hip(hipEventRecord(c->h2d_done[p], c->stream), "hipEventRecord"))) break;
    slot_used[p] = true;
    // a skipped file (status != 0) goes in as an empty file: no chunks
    const uint64_t* blens = lens + first;
    if (status) {
      skip_lens.assign(lens + first, lens + f);
      for (uint64_t i = first; i < f; i++)
        if (status[i]) skip_lens[i - first] = 0;
      blens = skip_lens.data();
    }
    rc = submit_batch(c, arena.p, f - first, offs.data(), blens, cut_ends, ids,
                      out_base + first, caps + first, sums ? sums + first : nullptr, budget);
    if (z.zout && rc == HBX_OK) jobs.push_back(ZJob{first, f - first, static_cast<const uint8_t*>(arena.p), offs});
    k++;
  }
  // collect everything in flight (also after a failure: the caller's arrays
  // must not be written once this call has returned); counted as waiting
  // for collection
  const double td = now();
  while (!c->pending.empty()) {
    const std::string keep = c->err;
    const int r2 = rc == HBX_OK ? collect() : wait_oldest(c);
    if (rc == HBX_OK) rc = r2;
    else c->err = keep;
  }
  // every compression job unpacked (also after a failure: the stages must be
  // idle before the arena ring is reused)
  while (!zq.empty()) {
    if (rc == HBX_OK) {
      rc = zdrain_one();
    } else {
      zq.front().fin.wait();  // its worker must be done before the stages and arenas go
      zq.pop_front();
    }
  }
  if (rc != HBX_OK && z.zout) zsync_all();
  c->io_s[1] += now() - td;
  if (z.zout && ab_env("HBX_ZDIAG"))
    std::fprintf(stderr, "zdiag: wait_oldest %.3f s, z_start %.3f s, z_finish %.3f s (event waits %.3f s), jobs %llu\n",
                 zt[0], zt[1], zt[2], zt[3], (unsigned long long)zjobs);
  return rc;
}
}  // namespace

int hbx_host_call_max(hbx_ctx* c, double ms[2], int reset) {
  if (!c || !ms) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  ms[0] = c->max_copy_ms;
  ms[1] = c->max_submit_ms;
  if (reset) c->max_copy_ms = c->max_submit_ms = 0.0;
  return HBX_OK;
}

int hbx_io_times(hbx_ctx* c, double s[3], int reset) {
  if (!c || !s) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  for (int i = 0; i < 3; i++) {
    s[i] = c->io_s[i];
    if (reset) c->io_s[i] = 0.0;
  }
  return HBX_OK;
}

int hbx_memcpy_h2d_async(hbx_ctx* c, void* d, const void* h, uint64_t n) {
  if (!c || (n && (!d || !h))) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HBX_TRY(c, hipSetDevice(c->device));
  const auto t0 = std::chrono::steady_clock::now();
  if (int frc = flush_input_wait(c)) return frc;
  g_slow.call("h2d: input wait", t0, c->launches);
  const auto t1 = std::chrono::steady_clock::now();
  HBX_TRY(c, hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, c->stream));
  c->max_copy_ms = std::max(c->max_copy_ms, ms_since(t1));
  g_slow.call("h2d: hipMemcpyAsync", t1, c->launches);
  return HBX_OK;
}

int hbx_input_after_oldest(hbx_ctx* c) {
  if (!c) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (c->broken) return c->fail(HBX_ERR_STATE, "context is unusable after a failed submit; destroy it");
  c->input_fence_set = false;
  if (c->pending.empty()) return HBX_OK;
  HBX_TRY(c, hipSetDevice(c->device));
  Batch* x = c->pending.front();
  // its last MD5 launch must have been issued: drain until it is (a caller
  // that reuses memory this early gets correct results, only slower)
  for (int k = 0; !x->finalized; k++) {
    const uint64_t l0 = c->launches;
    int rc = md5_step(c, kBudgetAll, true);
    if (rc) return rc;
    if (c->launches == l0 || k > 2) return c->fail(HBX_ERR_STATE, "drain launched nothing (internal)");
  }
  if (!x->joined || c->hstream == c->stream) return HBX_OK;  // (empty batch / one stream: in order already)
  // the completion event of the launch that finished it (or of a later one,
  // if that slot has been recorded again since)
  const uint64_t L = c->launches - x->final_launch <= kDoneRing ? x->final_launch : c->launches - 1;
  // (lean marks: nothing to enqueue once the host has seen it complete -- in
  // the steady state it finished two launches ago)
  if (c->lean_marks && hipEventQuery(c->order_free[L % kDoneRing]) == hipSuccess) return HBX_OK;
  c->input_fence_set = true;
  c->input_fence_L = L;
  if (c->lean_marks) {  // enqueued after the next plan (flush_input_wait), off the scan loop
    if (int frc = flush_input_wait(c)) return frc;  // (an earlier one not yet flushed goes first)
    c->input_wait_pending = true;
    c->input_wait_L = L;
    return HBX_OK;
  }
  HBX_TRY(c, hipStreamWaitEvent(c->stream, c->order_free[L % kDoneRing], 0));
  return HBX_OK;
}

int hbx_input_fence(hbx_ctx* c, void* stream) {
  if (!c) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (c->broken) return c->fail(HBX_ERR_STATE, "context is unusable after a failed submit; destroy it");
  HBX_TRY(c, hipSetDevice(c->device));
  if (int frc = flush_input_wait(c)) return frc;
  if (!stream || !c->input_fence_set) return HBX_OK;
  // Nothing to wait for once launch L is known complete.  The ring slot of L
  // is recorded again by launch L + kDoneRing: a fence called that late waits for
  // that later launch instead (issued after L on the same stream, so it
  // completes after L: conservative, never early).
  const uint64_t L = c->input_fence_L;
  hipEvent_t e = c->order_free[L % kDoneRing];
  if (L < c->k3_done_upto || hipEventQuery(e) == hipSuccess) {
    c->input_fence_set = false;
    return HBX_OK;
  }
  HBX_TRY(c, hipStreamWaitEvent(static_cast<hipStream_t>(stream), e, 0));
  return HBX_OK;
}

int hbx_after_stream(hbx_ctx* c, void* stream) {
  if (!c) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HBX_TRY(c, hipSetDevice(c->device));
  if (!stream) {
    // The null stream: a blocking scan stream (the CU-masked default) is
    // already ordered after prior null-stream work by the legacy default-
    // stream rule, on the GPU.  Recording an event on the null stream instead
    // would hold the host until the scan stream drains (measured: every
    // submit then waited for the previous batch's K1/K2, 0.3 ms hash-stream
    // gaps per step).
    unsigned flags = 0;
    HBX_TRY(c, hipStreamGetFlags(c->stream, &flags));
    if (!(flags & hipStreamNonBlocking)) return HBX_OK;
  }
  if (!c->producer) HBX_TRY(c, hipEventCreateWithFlags(&c->producer, hipEventDisableTiming));
  HBX_TRY(c, hipEventRecord(c->producer, static_cast<hipStream_t>(stream)));
  HBX_TRY(c, hipStreamWaitEvent(c->stream, c->producer, 0));  // every input read starts on the scan stream
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

// ---- block formats (hbx_formats.h) ----------------------------
uint64_t hbx_file_entry_size(const hbx_file_entry* e) { return e ? hbxfmt::entry_size(*e) : 0; }

int hbx_file_entry_serialize(const hbx_file_entry* e, uint8_t* out, uint64_t cap, uint64_t* n) {
  if (!e || (cap && !out) || (e->name_len && !e->name) || (e->link_len && !e->link && e->content_type == 4))
    return HBX_ERR_ARG;
  hbxfmt::Writer w{out, cap};
  hbxfmt::write_entry(w, *e);
  if (!w.ok) return HBX_ERR_CAPACITY;
  if (n) *n = w.n;
  return HBX_OK;
}

int hbx_file_entry_parse(const uint8_t* in, uint64_t len, hbx_file_entry* e, uint64_t* used) {
  if (!e || (len && !in)) return HBX_ERR_ARG;
  hbxfmt::Reader r{in, len};
  if (!hbxfmt::read_entry(r, *e).empty()) return HBX_ERR_FORMAT;
  if (used) *used = r.n;
  return HBX_OK;
}

int hbx_chain_block_serialize(const uint8_t* ids, const uint8_t* keys, uint32_t k, uint8_t* out,
                              uint64_t cap, uint64_t* n) {
  if ((k && !ids) || (cap && !out)) return HBX_ERR_ARG;
  hbxfmt::Writer w{out, cap};
  hbxfmt::write_chain(w, ids, keys, k);
  if (!w.ok) return HBX_ERR_CAPACITY;
  if (n) *n = w.n;
  return HBX_OK;
}

int hbx_chain_block_parse(const uint8_t* in, uint64_t len, uint32_t* k, uint8_t* ids, uint8_t* keys,
                          uint32_t cap) {
  if (!k || (len && !in)) return HBX_ERR_ARG;
  hbxfmt::Reader r{in, len};
  const uint32_t magic = r.u32();
  const uint32_t cnt = r.u32();
  if (!r.ok) return HBX_ERR_FORMAT;
  if (magic != hbxfmt::kMagicChain) return HBX_ERR_FORMAT;  // "corrupted FileChainBlock"
  *k = cnt;
  if ((uint64_t)cnt * 32ull > len - r.n) return HBX_ERR_FORMAT;
  if (cnt > cap && (ids || keys)) return HBX_ERR_CAPACITY;
  for (uint32_t i = 0; i < cnt && (ids || keys); i++) {
    const uint8_t* pair = r.take(32);
    if (ids) std::memcpy(ids + 16ull * i, pair, 16);
    if (keys) std::memcpy(keys + 16ull * i, pair + 16, 16);
  }
  return HBX_OK;
}

uint64_t hbx_directory_block_size(const hbx_file_entry* es, uint32_t n) {
  return (es || !n) ? hbxfmt::dir_size(es, n) : 0;
}

int hbx_directory_block_serialize(const hbx_file_entry* es, uint32_t n, uint8_t* out, uint64_t cap,
                                  uint64_t* n_out, uint8_t* links, uint32_t* n_links) {
  if ((n && !es) || (cap && !out)) return HBX_ERR_ARG;
  hbxfmt::Writer w{out, cap};
  const uint32_t nl = hbxfmt::write_dir(w, es, n, links);
  if (!w.ok) return HBX_ERR_CAPACITY;
  if (n_out) *n_out = w.n;
  if (n_links) *n_links = nl;
  return HBX_OK;
}

int hbx_directory_block_parse(const uint8_t* in, uint64_t len, hbx_file_entry* es, uint32_t cap,
                              uint32_t* n) {
  if (!n || (len && !in)) return HBX_ERR_ARG;
  hbxfmt::Reader r{in, len};
  const uint32_t magic = r.u32();
  const uint32_t cnt = r.u32();
  if (!r.ok || magic != hbxfmt::kMagicDir) return HBX_ERR_FORMAT;  // "corrupted DirectoryBlock"
  *n = cnt;
  for (uint32_t i = 0; i < cnt; i++) {
    hbx_file_entry tmp;
    if (!hbxfmt::read_entry(r, tmp).empty()) return HBX_ERR_FORMAT;
    if (es && i < cap) es[i] = tmp;
  }
  return (es && cnt > cap) ? HBX_ERR_CAPACITY : HBX_OK;
}

int hbx_directory_block_ids(hbx_ctx* c, uint32_t n_dirs, const hbx_file_entry* entries,
                            const uint64_t* entry_base, const uint32_t* n_entries, uint8_t* ids) {
  if (!c || (n_dirs && (!entries || !entry_base || !n_entries || !ids))) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->pending.empty()) return c->fail(HBX_ERR_STATE, "submitted batches are still pending");
  if (n_dirs == 0) return HBX_OK;
  HBX_TRY(c, hipSetDevice(c->device));
  // every directory block into one host image (256-B aligned, as hbx_verify_blocks
  // lays out its staging), one copy, one K6 launch
  std::vector<uint64_t> offs(n_dirs), lens(n_dirs), link_base(n_dirs);
  std::vector<uint32_t> nls(n_dirs);
  uint64_t total = 0, nlinks = 0;
  for (uint32_t d = 0; d < n_dirs; d++) {
    const hbx_file_entry* es = entries + entry_base[d];
    offs[d] = total;
    lens[d] = hbxfmt::dir_size(es, n_entries[d]);
    total += (lens[d] + 255) & ~uint64_t(255);
    link_base[d] = nlinks;
    for (uint32_t i = 0; i < n_entries[d]; i++) nlinks += hbxfmt::has_content(es[i].content_type) ? 1 : 0;
  }
  std::vector<uint8_t> img(total), links(16 * std::max<uint64_t>(nlinks, 1));
  for (uint32_t d = 0; d < n_dirs; d++) {
    hbxfmt::Writer w{img.data() + offs[d], lens[d]};
    nls[d] = hbxfmt::write_dir(w, entries + entry_base[d], n_entries[d], links.data() + 16 * link_base[d]);
    if (!w.ok) return c->fail(HBX_ERR_ARG, "directory " + std::to_string(d) + ": bad entry");
  }
  HBX_TRY(c, c->d_stage.ensure(total + 65536));
  uint8_t* arena = c->d_stage.as<uint8_t>();
  HBX_TRY(c, hipMemcpyAsync(arena, img.data(), total, hipMemcpyHostToDevice, c->stream));
  return verify_device(c, arena, n_dirs, offs.data(), lens.data(), links.data(), link_base.data(),
                       nls.data(), ids, nullptr, nullptr, nullptr);
}

// ---- zlib block compression (hbx_deflate.hip) -----------------
uint64_t hbx_deflate_bound(uint64_t len) {
  return 11ull + len + 5ull * ((len + hbxz::kSeg - 1) / hbxz::kSeg);
}

namespace {
// K7a -> K7s -> K7b over n blocks at device addresses src[i] (len[i] bytes,
// HBX_ARENA_SLACK readable after each) into device streams dst[i].
int deflate_device(hbx_ctx* c, uint64_t n, const uint64_t* src, const uint64_t* lens, const uint64_t* dst,
                   uint64_t* out_lens) {
  if (n == 0) return HBX_OK;
  if (n > 0xFFFFFFFFull) return c->fail(HBX_ERR_ARG, "too many blocks");
  std::vector<hbxz::ZBlock> zb(n);
  uint64_t nseg = 0;
  for (uint64_t i = 0; i < n; i++) {
    const uint64_t ns = (lens[i] + hbxz::kSeg - 1) / hbxz::kSeg;
    zb[i] = hbxz::ZBlock{src[i], dst[i], lens[i], (uint32_t)nseg, (uint32_t)ns};
    nseg += ns;
    if (nseg > 0x7FFFFFFFull) return c->fail(HBX_ERR_ARG, "too much data in one call");
  }
  hipStream_t s = c->stream;
  HBX_TRY(c, c->d_zblk.ensure(n * sizeof(hbxz::ZBlock)));
  HBX_TRY(c, c->d_zinfo.ensure(std::max<uint64_t>(nseg, 1) * sizeof(hbxz::SegInfo)));
  HBX_TRY(c, c->d_zoff.ensure(std::max<uint64_t>(nseg, 1) * 8));
  HBX_TRY(c, c->d_zlen.ensure(n * 8));
  HBX_TRY(c, c->d_zimg.ensure(std::max<uint64_t>(nseg, 1) * hbxz::kSlot));
  HBX_TRY(c, hipMemcpyAsync(c->d_zblk.p, zb.data(), n * sizeof(hbxz::ZBlock), hipMemcpyHostToDevice, s));
  const hbxz::ZBlock* dz = c->d_zblk.as<hbxz::ZBlock>();
  if (nseg) {
    hipLaunchKernelGGL(hbx_k7_deflate_entropy, dim3((uint32_t)nseg), dim3(hbxz::kEThreads), 0, s, dz, (uint32_t)n,
                       (uint32_t)nseg, c->d_zinfo.as<hbxz::SegInfo>());
    hipLaunchKernelGGL(hbx_k7_deflate_size, dim3((uint32_t)nseg), dim3(hbxz::kThreads), 0, s, dz, (uint32_t)n,
                       (uint32_t)nseg, c->d_zinfo.as<hbxz::SegInfo>(), c->d_zimg.as<uint32_t>());
    hipLaunchKernelGGL(hbx_k7_deflate_code, dim3((uint32_t)nseg), dim3(hbxz::kThreads), 0, s, dz, (uint32_t)n,
                       (uint32_t)nseg, c->d_zinfo.as<hbxz::SegInfo>(), c->d_zimg.as<uint32_t>());
    HBX_TRY(c, hipGetLastError());
  }
  hipLaunchKernelGGL(hbx_k7_deflate_plan, dim3((uint32_t)n), dim3(64), 0, s, dz, (uint32_t)n,
                     c->d_zinfo.as<hbxz::SegInfo>(), c->d_zoff.as<uint64_t>(), c->d_zlen.as<uint64_t>());
  HBX_TRY(c, hipGetLastError());
  if (nseg) {
    hipLaunchKernelGGL(hbx_k7_deflate_write, dim3((uint32_t)nseg), dim3(hbxz::kWThreads), 0, s, (uint32_t)nseg,
                       c->d_zinfo.as<hbxz::SegInfo>(), c->d_zimg.as<uint32_t>(), c->d_zoff.as<uint64_t>(), dz,
                       (uint32_t)n);
    HBX_TRY(c, hipGetLastError());
  }
  HBX_TRY(c, hipMemcpyAsync(out_lens, c->d_zlen.p, n * 8, hipMemcpyDeviceToHost, s));
  HBX_TRY(c, hipStreamSynchronize(s));
  return HBX_OK;
}
}  // namespace

int hbx_deflate_blocks_device(hbx_ctx* c, const void* d_arena, uint64_t n, const uint64_t* offs,
                              const uint64_t* lens, void* d_out, const uint64_t* out_offs,
                              const uint64_t* out_caps, uint64_t* out_lens) {
  if (!c || (n && (!d_arena || !offs || !lens || !d_out || !out_offs || !out_caps || !out_lens)))
    return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->pending.empty()) return c->fail(HBX_ERR_STATE, "submitted batches are still pending");
  HBX_TRY(c, hipSetDevice(c->device));
  std::vector<uint64_t> src(n), dst(n);
  for (uint64_t i = 0; i < n; i++) {
    if (out_caps[i] < hbx_deflate_bound(lens[i]))
      return c->fail(HBX_ERR_CAPACITY, "output capacity below hbx_deflate_bound for block " + std::to_string(i));
    src[i] = reinterpret_cast<uint64_t>(d_arena) + offs[i];
    dst[i] = reinterpret_cast<uint64_t>(d_out) + out_offs[i];
  }
  return deflate_device(c, n, src.data(), lens, dst.data(), out_lens);
}

int hbx_deflate_blocks(hbx_ctx* c, uint64_t n, const uint8_t* const* datas, const uint64_t* lens,
                       uint8_t* const* outs, const uint64_t* caps, uint64_t* out_lens) {
  if (!c || (n && (!datas || !lens || !outs || !caps || !out_lens))) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->pending.empty()) return c->fail(HBX_ERR_STATE, "submitted batches are still pending");
  if (n == 0) return HBX_OK;
  HBX_TRY(c, hipSetDevice(c->device));
  std::vector<uint64_t> soff(n), doff(n), src(n), dst(n);
  uint64_t sin = 0, sout = 0;
  for (uint64_t i = 0; i < n; i++) {
    if (lens[i] && !datas[i]) return c->fail(HBX_ERR_ARG, "null block data");
    if (caps[i] < hbx_deflate_bound(lens[i]))
      return c->fail(HBX_ERR_CAPACITY, "output capacity below hbx_deflate_bound for block " + std::to_string(i));
    soff[i] = sin;
    sin += (lens[i] + 255) & ~uint64_t(255);
    doff[i] = sout;
    sout += (hbx_deflate_bound(lens[i]) + 15) & ~uint64_t(15);
  }
  HBX_TRY(c, c->d_stage.ensure(sin + 65536));
  HBX_TRY(c, c->d_zout.ensure(sout + 64));
  uint8_t* arena = c->d_stage.as<uint8_t>();
  uint8_t* zo = c->d_zout.as<uint8_t>();
  for (uint64_t i = 0; i < n; i++) {
    if (lens[i]) HBX_TRY(c, hipMemcpyAsync(arena + soff[i], datas[i], lens[i], hipMemcpyHostToDevice, c->stream));
    src[i] = reinterpret_cast<uint64_t>(arena + soff[i]);
    dst[i] = reinterpret_cast<uint64_t>(zo + doff[i]);
  }
  const int rc = deflate_device(c, n, src.data(), lens, dst.data(), out_lens);
  if (rc) return rc;
  std::vector<uint8_t> host(sout);
  HBX_TRY(c, hipMemcpy(host.data(), zo, sout, hipMemcpyDeviceToHost));
  for (uint64_t i = 0; i < n; i++) std::memcpy(outs[i], host.data() + doff[i], out_lens[i]);
  return HBX_OK;
}

// ---- wire protocol framing (hbx_wire.h) -----------------------
int hbx_wire_encode_id(uint16_t num, uint32_t type, const uint8_t id[16], uint8_t out[22]) {
  if (!id || !out || !hbxwire::is_id_msg(type)) return HBX_ERR_ARG;
  hbxfmt::Writer w{out, 22};
  const uint8_t nb[2] = {(uint8_t)(num >> 8), (uint8_t)num};
  w.bytes(nb, 2);
  w.u32(type);
  w.bytes(id, 16);
  return w.ok ? HBX_OK : HBX_ERR_CAPACITY;
}

int hbx_wire_encode_block_header(uint16_t num, uint32_t type, const uint8_t id[16], const uint8_t* links,
                                 uint32_t n_links, uint8_t data_type, uint32_t data_len, uint8_t* out,
                                 uint64_t cap, uint64_t* n) {
  if (!id || (n_links && !links) || (cap && !out) || !hbxwire::is_block_msg(type)) return HBX_ERR_ARG;
  hbxfmt::Writer w{out, cap};
  const uint8_t nb[2] = {(uint8_t)(num >> 8), (uint8_t)num};
  w.bytes(nb, 2);
  w.u32(type);
  w.bytes(id, 16);  // HashboxBlock.Serialize, block.go:56-69
  w.u32(n_links);
  w.bytes(links, 16ull * n_links);
  w.u8(data_type);
  w.u32(data_len);
  if (!w.ok) return HBX_ERR_CAPACITY;
  if (n) *n = w.n;
  return HBX_OK;
}

int hbx_wire_parse(const uint8_t* in, uint64_t len, hbx_wire_msg* msg) {
  if (!msg || (len && !in)) return HBX_ERR_ARG;
  return hbxwire::parse(in, len, msg);
}

int hbx_verify_submit_device(hbx_ctx* c, const void* d_arena, uint64_t n, const uint64_t* offs,
                             const uint64_t* lens, const uint8_t* links, const uint64_t* link_base,
                             const uint32_t* n_links, uint8_t* ids, const uint8_t* expect, uint8_t* ok,
                             uint64_t* n_bad) {
  if (!c || (n && (!d_arena || !offs || !lens))) return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HBX_TRY(c, hipSetDevice(c->device));
  if (n_bad) *n_bad = 0;
  return submit_verify(c, static_cast<const uint8_t*>(d_arena), n, offs, lens, links, link_base, n_links, ids,
                       expect, ok, n_bad, c->md5_slice ? c->md5_slice : kBudgetAll);
}

// ---- zlib inflate (hbx_inflate.hip) -----------------------------------------
int hbx_inflate_blocks_device(hbx_ctx* c, const void* d_in, uint64_t n, const uint64_t* in_offs,
                              const uint64_t* in_lens, void* d_out, const uint64_t* out_offs,
                              const uint64_t* out_caps, uint64_t* out_lens, uint32_t* status) {
  if (!c || (n && (!d_in || !in_offs || !in_lens || !d_out || !out_offs || !out_caps || !out_lens || !status)))
    return HBX_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->pending.empty()) return c->fail(HBX_ERR_STATE, "submitted batches are still pending");
  if (n == 0) return HBX_OK;
  if (n > 0x7FFFFFFFull) return c->fail(HBX_ERR_ARG, "too many streams");
  HBX_TRY(c, hipSetDevice(c->device));
  // one wave per stream, longest first (the long ones start first)
  std::vector<uint32_t> perm(n);
  for (uint64_t i = 0; i < n; i++) {
    if (in_lens[i] > 0xFFFFFFFFull || out_caps[i] > 0xFFFFFFFFull) return c->fail(HBX_ERR_ARG, "stream too large");
    perm[i] = (uint32_t)i;
  }
  std::stable_sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t b) { return in_lens[a] > in_lens[b]; });
  // a wave per stream, except for tens of thousands of short compressible
  // streams, where 64 streams per wave (one per lane) keep more streams in
  // flight, and for long compressible streams when few of them fill the GPU:
  // those are split into regions decoded in parallel (hbx_inflate_split.hip).
  // HBX_K8_MODE=lane|wave|split forces one (tests; split then takes every
  // stream of >= 2 regions, compressible or not).
  uint64_t tin = 0, tcap = 0;
  for (uint64_t i = 0; i < n; i++) {
    tin += in_lens[i];
    tcap += out_caps[i];
  }
  bool lanes = n >= 8192 && tin * 10 < tcap * 7 && tcap / n <= (256u << 10);
  const char* mode = ab_env("HBX_K8_MODE");
  if (mode) lanes = std::strcmp(mode, "lane") == 0;
  const bool force_split = mode && std::strcmp(mode, "split") == 0;
  const bool no_split = lanes || (mode && std::strcmp(mode, "wave") == 0);
  auto splits = [&](uint32_t i) {
    if (no_split || in_lens[i] < 2ull * hbxs::kSplitRegion) return false;
    return force_split || in_lens[i] * 10 < out_caps[i] * 8;
  };
  // Scratch of one split stream: regions of kSplitRegion compressed bytes,
  // each with room for twice its share of the stream's output capacity in
  // 16-bit symbols, at most kSplitSymCap (a region that needs more overflows
  // and the stream is inflated again by the wave kernel).
  constexpr uint64_t kSplitSymCap = 4ull << 20;
  auto region_syms = [&](uint64_t len, uint64_t cap, uint32_t& cnt) {
    cnt = (uint32_t)((len + hbxs::kSplitRegion - 1) / hbxs::kSplitRegion);
    const uint64_t share = (2ull * cap + cnt - 1) / cnt;
    return std::min<uint64_t>(((share + 63) & ~63ull) + 4096, kSplitSymCap);
  };
  uint64_t long_streams = 0;
  for (uint64_t i = 0; i < n; i++) long_streams += splits(perm[i]) ? 1 : 0;
  // enough streams to fill the SIMDs on their own: no split (it costs a
  // second pass over 2 bytes per output byte)
  bool split_any = long_streams > 0 && (force_split || long_streams < 2048);
  // The split path's scratch has a budget (a quarter of the free device
  // memory, at most 16 GiB): the longest candidates take it in order, the
  // rest go to the wave kernel, which needs no scratch (advisor r04).
  std::vector<uint8_t> take(n, 0);
  if (split_any) {
    size_t fr = 0, tot = 0;
    uint64_t budget = 256ull << 20;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) budget = std::max<uint64_t>(budget, std::min<uint64_t>(fr / 4, 16ull << 30));
    uint64_t used = 0;
    long_streams = 0;
    for (uint64_t k = 0; k < n; k++) {
      const uint32_t i = perm[k];
      if (!splits(i)) continue;
      uint32_t cnt = 0;
      const uint64_t syms = region_syms(in_lens[i], out_caps[i], cnt);
      const uint64_t b = 2ull * syms * cnt;  // scratch bytes of its regions
      if (used + b > budget) continue;
      used += b;
      take[i] = 1;
      long_streams++;
    }
    split_any = long_streams > 0;
  }
  // split streams last, so the wave kernel takes the prefix [0, nw)
  if (split_any)
    std::stable_partition(perm.begin(), perm.end(), [&](uint32_t i) { return !take[i]; });
  uint64_t nw = split_any ? n - long_streams : n;
  std::vector<InflateDesc> desc(n);
  for (uint64_t k = 0; k < n; k++) {
    const uint32_t i = perm[k];
    desc[k].src = reinterpret_cast<uint64_t>(d_in) + in_offs[i];
    desc[k].dst = reinterpret_cast<uint64_t>(d_out) + out_offs[i];
    desc[k].len = (uint32_t)in_lens[i];
    desc[k].cap = (uint32_t)out_caps[i];
  }
  hipStream_t s = c->stream;
  HBX_TRY(c, c->d_idesc.ensure(n * sizeof(InflateDesc)));
  HBX_TRY(c, c->d_ires.ensure(n * 8));
  // The region table and every split buffer exist before the first kernel is
  // queued: a failure then leaves nothing running, and an allocation that
  // fails sends those streams to the wave kernel instead of failing the call.
  std::vector<SplitRegion> reg;
  std::vector<uint32_t> meta;
  if (split_any) {
    meta.assign(3 * (n - nw), 0u);
    uint64_t sym = 0;
    for (uint64_t k = nw; k < n; k++) {
      uint32_t cnt = 0;
      const uint32_t scap = (uint32_t)region_syms(desc[k].len, desc[k].cap, cnt);
      meta[k - nw] = (uint32_t)k;
      meta[(n - nw) + (k - nw)] = (uint32_t)reg.size();
      meta[2 * (n - nw) + (k - nw)] = cnt;
      const uint32_t first = (uint32_t)reg.size();
      for (uint32_t r = 0; r < cnt; r++) {
        reg.push_back(SplitRegion{(uint32_t)k, r, first, cnt, sym, scap, 0u});
        sym += scap;
      }
    }
    const uint64_t nreg = reg.size();
    bool ok = nreg <= 0x7FFFFFFFull;
    for (auto [buf, bytes] : {std::pair<DevBuf*, uint64_t>{&c->d_sreg, nreg * sizeof(SplitRegion)},
                              {&c->d_sstart, nreg * 8}, {&c->d_sres, nreg * sizeof(SplitResult)},
                              {&c->d_sscratch, sym * 2 + 64}, {&c->d_smeta, meta.size() * 4}})
      if (ok && buf->ensure(bytes) != hipSuccess) {
        (void)hipGetLastError();  // the failed allocation is not an error of this call
        ok = false;
      }
    if (!ok) {  // every stream to the wave kernel
      split_any = false;
      nw = n;
    }
  }
  HBX_TRY(c, hipMemcpyAsync(c->d_idesc.p, desc.data(), n * sizeof(InflateDesc), hipMemcpyHostToDevice, s));
  uint32_t* dres = c->d_ires.as<uint32_t>();
  const InflateDesc* ddesc = c->d_idesc.as<InflateDesc>();
  if (nw && lanes)
    hipLaunchKernelGGL(hbx_k8_inflate_lanes, dim3((uint32_t)((nw + 63) / 64)), dim3(64), 0, s, ddesc, (uint32_t)nw,
                       dres, dres + n);
  else if (nw)
    hipLaunchKernelGGL(hbx_k8_inflate, dim3((uint32_t)nw), dim3(64), 0, s, ddesc, (uint32_t)nw, dres, dres + n);
  HBX_TRY(c, hipGetLastError());
  if (split_any) {
    const uint64_t nreg = reg.size(), ns = n - nw;
    HBX_TRY(c, hipMemcpyAsync(c->d_sreg.p, reg.data(), nreg * sizeof(SplitRegion), hipMemcpyHostToDevice, s));
    HBX_TRY(c, hipMemcpyAsync(c->d_smeta.p, meta.data(), meta.size() * 4, hipMemcpyHostToDevice, s));
    const SplitRegion* dreg = c->d_sreg.as<SplitRegion>();
    uint64_t* dstart = c->d_sstart.as<uint64_t>();
    SplitResult* dsres = c->d_sres.as<SplitResult>();
    const uint32_t* dmeta = c->d_smeta.as<uint32_t>();
    hipLaunchKernelGGL(hbx_k8s_find, dim3((uint32_t)nreg), dim3(64), 0, s, ddesc, dreg, (uint32_t)nreg, dstart);
    hipLaunchKernelGGL(hbx_k8s_decode, dim3((uint32_t)nreg), dim3(64), 0, s, ddesc, dreg, (uint32_t)nreg,
                       static_cast<const uint64_t*>(dstart), c->d_sscratch.as<uint16_t>(), dsres);
    hipLaunchKernelGGL(hbx_k8s_resolve, dim3((uint32_t)ns), dim3(256), 0, s, ddesc, dmeta, dmeta + ns, dmeta + 2 * ns,
                       (uint32_t)ns, dreg, static_cast<const uint64_t*>(dstart),
                       static_cast<const SplitResult*>(dsres), static_cast<const uint16_t*>(c->d_sscratch.as<uint16_t>()),
                       dres, dres + n);
    HBX_TRY(c, hipGetLastError());
  }
  std::vector<uint32_t> res(2 * n);
  HBX_TRY(c, hipMemcpyAsync(res.data(), dres, n * 8, hipMemcpyDeviceToHost, s));
  HBX_TRY(c, hipStreamSynchronize(s));
  if (split_any) {  // the streams the split path did not resolve: the wave kernel, from scratch
    std::vector<InflateDesc> again;
    std::vector<uint64_t> at;
    for (uint64_t k = nw; k < n; k++)
      if (res[n + k] != 0u) {
        again.push_back(desc[k]);
        at.push_back(k);
      }
    c->k8_split_fallbacks += again.size();
    c->k8_split_streams += n - nw;
    if (!again.empty()) {
      const uint64_t m = again.size();
      HBX_TRY(c, hipMemcpyAsync(c->d_idesc.p, again.data(), m * sizeof(InflateDesc), hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(hbx_k8_inflate, dim3((uint32_t)m), dim3(64), 0, s, ddesc, (uint32_t)m, dres, dres + m);
      HBX_TRY(c, hipGetLastError());
      std::vector<uint32_t> r2(2 * m);
      HBX_TRY(c, hipMemcpyAsync(r2.data(), dres, m * 8, hipMemcpyDeviceToHost, s));
      HBX_TRY(c, hipStreamSynchronize(s));
      for (uint64_t q = 0; q < m; q++) {
        res[at[q]] = r2[q];
        res[n + at[q]] = r2[m + q];
      }
    }
  }
  for (uint64_t k = 0; k < n; k++) {
    out_lens[perm[k]] = res[k];
    status[perm[k]] = res[n + k];
  }
  // the split scratch is not kept past the call once it is large (the stream
  // is idle here: everything above was synchronized)
  if (c->d_sscratch.cap > (256ull << 20)) c->d_sscratch.release();
  return HBX_OK;
}

}  // extern "C"
